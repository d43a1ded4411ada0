// mz_internal.h — shared declarations of the libmz HIP engine (gfx950).
//
// The three FC networks (Learning.jl:87-142) are executed as "plans": a plan
// is a list of stages separated by workgroup barriers; a stage is a list of
// tasks; a task is one 16-row output block of one Dense layer, computed by
// one wavefront as a 16 (outputs) x 16 (games/samples) tile with f32 MFMA
// (v_mfma_f32_16x16x4_f32).  Activations live in LDS as [rows][16] f32
// (row = feature, column = game of the workgroup's tile).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mz.h"
#include "../../include/mz_detmath.h"

#pragma clang fp contract(off)

#define MZ_TILE 16          // games (or samples) per workgroup tile = MFMA N
#define MZ_THREADS 256      // 4 wavefronts
#ifndef MZ_L2_BLOCKS         // (-D override: timing A/B builds only; the oracle's order is NB below)
#define MZ_L2_BLOCKS 128    // Σθ² / ∇ (/ fused ADAM) blocks per net in mz_learner_grad_kernel* (oracle ora_sqnorm: NB)
#endif
#define MZ_MAX_STAGES 64

// Device fault word (mz_handle d_fault): bits set by a kernel that gave up
// waiting for another workgroup's publish; the host reads it at its next
// synchronisation (every host-synchronous call and mz_sync), clears it and
// fails that call with a message (mz_last_error) — a producer that never
// publishes is reported, never silently consumed as stale data.
enum { MZ_FAULT_RS_TRUNK = 1,      // mz_rsearch_nets: the dynamics workgroup's trunk publish
       MZ_FAULT_RD_PROGRESS = 2 }; // mz_runroll_fused_r: a chain block's h_s / trunk publish
#define MZ_POLL_TICKS 200000000ull // 2 s of the 100 MHz s_memrealtime clock

// One lane polls a 64-bit progress word (relaxed, agent scope) until it
// reaches `want`, sleeping between loads; after `ticks` of the constant clock
// it ORs `code` into *fault and returns false (the caller still drains, so the
// grid exits).  The payload is stored write-through (agent-scope atomic
// stores), drained by every storing wave (vmcnt 0) before the barrier that
// precedes the flag store, and read with agent-scope loads: the R1 hand-off
// of cdna_hip_programming.md Guideline 16, which needs no release fence; the
// wavefront-scope acquire after the poll only keeps the compiler from moving
// the payload loads above it.
__device__ __forceinline__ bool mz_poll_ge(const unsigned long long* w, unsigned long long want, unsigned* fault,
                                           unsigned code, unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            if (fault) __hip_atomic_fetch_or(fault, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return ok;
}

// One Dense layer inside a plan.  All offsets are in floats.
struct LayerDesc {
    int w_off;     // packed weights: [n_ob][4*nq k-steps][64 lanes]
    int b_off;     // packed bias: [n_ob*16]
    int nq;        // k-steps per quarter (= ceil(K/16)); kq = 4*nq k values
    int n_ob;      // output blocks of 16 rows
    int act;       // MZ_ACT_*
    int in_off;    // LDS activation input  [16*nq*4 rows][16]
    int out_off;   // LDS activation output [n_ob*16 rows][16]
    int out_rows;  // real outputs
    int bn;        // make_dense with use_batch_norm: BatchNorm(out, relu) after the affine;
                   // γ at b_off + n_ob*16, β at b_off + 2*n_ob*16 of the packed bias image
};

// Flux BatchNorm in test mode (μ = 0, σ² = 1, ϵ = 1f-5, the reference's
// never-updated running statistics): γ·((t − 0)/√(1 + ϵ)) + β, IEEE division
// by the f32 √(1 + 1f-5) (0x3f80002a), as the oracle's bn_apply.
#define MZ_BN_S 0x1.000054p+0f
__host__ __device__ __forceinline__ float mz_bn_apply(float t, float g, float b) {
    const float xh = (t - 0.0f) / MZ_BN_S;
    return g * xh + b;
}

// Device plan image (int array):
//   [0] n_stages, [1] n_layers, [2] n_tasks,
//   [3 .. 3+n_stages]            stage_begin (n_stages+1 entries),
//   then n_tasks x {layer, ob},  then n_layers x LayerDesc.
struct PlanView {
    int n_stages, n_layers, n_tasks;
    const int* stage_begin;
    const int* tasks;
    const LayerDesc* layers;
};

__device__ __forceinline__ PlanView plan_view(const int* p) {
    PlanView v;
    v.n_stages = p[0]; v.n_layers = p[1]; v.n_tasks = p[2];
    v.stage_begin = p + 3;
    v.tasks = v.stage_begin + v.n_stages + 1;
    v.layers = reinterpret_cast<const LayerDesc*>(v.tasks + 2 * v.n_tasks);
    return v;
}

// LDS region offsets of the standard activation layout (floats); the host
// fills this and passes it by value.
struct ActLayout {
    int x_rep, x_pred, x_dyn;     // inputs: stacked obs, hidden, state-action
    int h_out, v_out, p_out, r_out;
    int rows_rep, rows_pred, rows_dyn;   // padded input rows (zeroed)
    int v_act, r_act;             // activations of the value / reward output layers (applied at read-out)
    int total;                    // floats
};

// Search-kernel parameters (passed by value).
struct SearchParams {
    int G, S, A, H, players, obs_feat;     // obs_feat = stacked features
    int plane;                             // W*H of the board (action plane size)
    int exploration;
    uint32_t rng_step, game_offset;
    uint64_t seed;
    float temperature, discount, dirichlet_alpha, exploration_eps;
    const float* temp_g;   // per-game temperatures (self-play temperature_threshold) or NULL
    // inputs
    const float* obs; const uint8_t* legal; const int32_t* to_play;
    // outputs
    float* child_visits; float* root_value; int32_t* action_out;
    // model
    const float* Wp; const float* Bp;
    const int* plan_root; const int* plan_sim;
    const int* plan_sim_res;  // register-resident image of plan_sim (NULL: not eligible)
    ActLayout lay;
    // tables (host-computed with libm so the oracle matches bit-exactly)
    const double* pbc_tab;    // log2((N + base + 1)/base) + c_init, N = 0..S+1
    const double* sqrt_tab;   // sqrt(N), N = 0..S+1
    const float* aval_tab;    // Float32(a / |A|), a = 1..A
    // tree storage in HBM: per game tree_game_bytes (mz_tree_device.h layout);
    // the working copy when the tree does not fit in LDS, else the debug dump
    char* tree;
    size_t tree_game_bytes;
    int dump_tree;            // LDS-tree kernel: copy the final tree to `tree`
    float* hid;               // hidden states [G][S+1][H]
    unsigned long long* stamps;   // diagnostic build (-DMZ_STAMPS) only: [grid][8] cycles
};

// Learner unroll-kernel parameters.
struct UnrollParams {
    int B, K, A, H, plane, obs_feat;
    const float* obs;        // (obs_feat, B)
    const float* actions;    // (K+1, B) float action ids
    float* pv;               // (K+1, B) predicted values
    float* pp;               // (A, K+1, B) predicted policies (probabilities)
    float* pr;               // (K+1, B) predicted rewards
    const float* Wp; const float* Bp;
    const int* plan_repr; const int* plan_sim;
    ActLayout lay;
};

// ADAM state and image scatter maps for mz_adam_kernel / the fused update of
// mz_learner_grad_kernel* (on = 1: update in place with G = 2θ, world = 1).
struct LgAdam {
    int on;
    float* M; float* V;
    double bp1, bp2, eta;
    float* Wp; float* Bp; const int* inv_tile; float* smw; float* smb; const int* inv_small;
};

__host__ __device__ inline int mz_round16(int x) { return (x + 15) & ~15; }
