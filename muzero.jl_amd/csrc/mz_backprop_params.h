// mz_backprop_params.h — the corrected-gradient learner (MZ_LEARN_CORRECTED):
// real backpropagation through the K-step unroll of the FC nets.
//
// The reference differentiates only sum(sqnorm, params) (quirk Q11: the
// predictions are computed outside the Zygote.pullback closures,
// Learning.jl:347-393), so every gradient is 2θ.  The corrected mode
// differentiates the loss it meant to (Learning.jl:261-288) through the same
// forward (Q10 alignment, make_dynamics_input's 2h, :293-304), as a
// per-sample mean so a data-parallel all-reduce-mean equals the global batch:
//   L = (1/B) Σ_b (w_b / g_b) [ Σ_{k=0..K} (v_bk − z_bk)²
//                              + Σ_{k=0..K} CE(ℓ_bk, π_bk)
//                              + intermediate_rewards · Σ_{k=1..K} (r_bk − u_bk)² ]
//       + Σθ²
// with v = tanh(value head), ℓ the policy head's logits (logitcrossentropy
// on logits, not on the softmax of a softmax, Q3), r the reward head after
// reward_activation, w the PER weights (1 without PER), g gradient_scale.
//
// The unrolled graph is a host-built list of layer applications on tiles of
// 16 samples (one MFMA N-tile): dense layers y = act(W x + b) and the
// concatenation sa = [2h ; a/|A| plane].  Activations and gradients live in
// per-tile arenas in HBM ([rows][16] f32 per tensor).
#pragma once
#include <stdint.h>

enum { BP_DENSE = 0, BP_CONCAT = 1 };
enum { BP_HEAD_V = 0, BP_HEAD_P = 1, BP_HEAD_R = 2 };

struct BpApp {
    int op;               // BP_DENSE / BP_CONCAT
    int w_off, b_off;     // dense: flat offsets of W (out,in) column-major and b
    int in, out, act;     // dense: dims, activation; concat: in = H (hidden), out = H + plane
    int x, y;             // arena offsets (floats) of the input / output tensor
    int step;             // concat: action column k (actions[b][k]); dense: layer id
    // mz_bp_tile_lv's LDS tensor cache (float offsets into it, -1: the arena
    // only): the forward input / output copies, the backward ∂L/∂y copy (written
    // out to the arena when read) and the ∂L/∂x accumulator; gxf = 1 on the
    // tensor's first contribution (the zeroed arena's sum starts there)
    int xs, ys, gys, gxs, gxf;
    // make_dense with use_batch_norm (Learning.jl:70-78): the test-mode
    // BatchNorm γ·(t/√(1+ε)) + β between the Dense and its relu; β at bn_off,
    // γ at bn_off + out (-1: none), t = W x + b kept in the arena at z for mz_bp_dw
    int bn_off, z;
};

struct BpHead {
    int kind;             // BP_HEAD_V / P / R
    int y;                // arena offset of the head's output tensor
    int step;             // unroll step k (targets column)
};

struct BpUse { int x, y, z; };   // one application of a dense layer: input / output / pre-BatchNorm t arena offsets

struct BpLayer {
    int w_off, b_off, in, out, act;
    int bn_off;           // β at bn_off, γ at bn_off + out (-1: no BatchNorm)
    int use0, n_use;      // uses[use0 .. use0 + n_use)
};

struct BpJob { int layer, ob, ib; };   // one 16x16 block of dW (ib = -1: the bias block of row block ob)

struct BpParams {
    int B, K, A, H, plane, obs_feat, tile_floats, n_app, n_head, obs_t, intermediate_rewards;
    const BpApp* apps; const BpHead* heads;
    float* act; float* grad;              // arenas [tiles][tile_floats]
    const float* flat;
    const float* obs; const float* actions; const float* tv; const float* tr; const float* tp;
    const float* gscale; const float* weights;
    float* terms;                         // [B][K+1][3]: (v−z)², CE, (r−u)²
    float* pv; float* pp; float* pr;      // the read-outs (K+1,B) / (A,K+1,B) / (K+1,B), as the unroll's
    // level schedule (mz_bp_tile_lv): the forward / backward applications
    // grouped into dependency levels, each a list of units {app, block} — a
    // dense layer's 16-row output block (forward) or 16-row input block
    // (backward dX), or a whole concatenation (block 0); lev[l] .. lev[l+1]
    int n_flev, n_blev, n_funit, n_bunit;
    const int2* funits; const int* flev;
    const int2* bunits; const int* blev;
    const int* fsync; const int* bsync;   // per level: 1 = the barrier after it drains the arena stores
    int cache_floats, obs_s;              // the LDS tensor cache (0: none); the observation's copy (-1: none)
    int nflat;                            // mz_bp_tile_lv warms the workgroup's L2 with the parameters (all levels read them)
    unsigned long long* stamps;           // diagnostic build (-DMZ_STAMPS) only: level end cycles of tile 0
};
#ifndef BP_LV_THREADS
#define BP_LV_THREADS 1024                // mz_bp_tile_lv: 16 waves, a unit per wave per level
#endif
#ifndef BP_LV_LDS
#define BP_LV_LDS 1                       // the schedule and descriptors staged in LDS
#endif
#ifndef BP_LV_SIMPLE
#define BP_LV_SIMPLE 1                    // units run as bp_dense_*_blk (operands loaded in the unit)
#endif
#ifndef BP_LV_PREFETCH
#define BP_LV_PREFETCH 0                  // the next level's unit, weights and bias loaded before each barrier
                                          // (measured slower: 1.91k vs 2.29k steps/s, tools/ab_corrected.sh)
#endif

struct BpDwParams {
    int tiles, tile_floats, n_job;
    const BpJob* jobs; const BpLayer* layers; const BpUse* uses;
    const float* act; const float* grad; const float* flat;
    float* out;                           // Flux-order data term of the gradient (2θ: mz_adam_kernel)
    double* sq;                           // [n_job]: Σθ² of each job's parameter block (f64, fixed order)
};

struct BpFoldParams {
    int B, K;
    const float* terms; const float* gscale; const float* weights;
    const float* flat; const size_t* netoff;
    float* losses;                        // {value, reward, policy, Σθ² repr, pred, dyn}
    const double* sq; int job0[4];        // mz_bp_dw's per-job Σθ²; jobs [job0[n], job0[n+1]) are net n's
};

// ---- the corrected learner for the ResNet nets (mz_rbp_sample / mz_rbp_dw)
// mz_rbp_sample, one workgroup per sample: the unroll's list of applications
// on that sample's arena in HBM (conv tensors [channel][position], f = p + P·c,
// the Flux.flatten order; dense vectors [feature]), the heads, then the list in
// reverse for the input gradients.  Convs run as 16x16 f32 MFMA blocks (rows =
// output channels, columns = board positions; the operand of a k×k conv is
// gathered through the kernel taps, Flux's flipped cross-correlation, zero off
// the board); BatchNorm is the test-mode affine γ·(t/√(1+ε)) + β; a block's
// second conv adds the saved input before its relu.  The arenas keep every
// application's output y, its pre-BatchNorm t and ∂L/∂y, so the parameter
// gradients need no per-sample copy: mz_rbp_dw gives each 16x16 block of a
// layer's dW (and each 16-channel block of db, dβ, dγ) one wave, which sums
// over (sample, application of the layer, position) — the K dimension of its
// MFMAs — with ∂L/∂t re-formed from the arenas as the operand is loaded.  The
// result is the data term (mz_adam_kernel adds 2θ).
enum { RBP_CONV = 0, RBP_DENSE = 1, RBP_CONCAT = 2 };

struct RbpApp {
    int op;
    int w_off, b_off, bn_off;   // flat offsets; bn_off: β at bn_off, γ at bn_off + cout (-1: no BatchNorm)
    int cin, cout, kw, kh, act; // conv: channels and kernel; dense: in, out
    int x, y, z, res;           // arena offsets: input, output (after the activation), the conv's t = Wx + b
                                // (BatchNorm layers), the residual input (-1: none)
    int step;                   // concat: action column; conv / dense: 1 = no input gradient (the observation)
    int xb, rb, yb;             // forward LDS ring slots (mz_rbp_sample) of x, res (-1: read from the arena), y
    int fsync;                  // 1: the barrier after this application drains the arena stores (a later
                                // one reads the arena); else an LDS-only barrier
    // backward LDS ring: the slot holding ∂L/∂y (gyb; written out to the arena
    // when read), the slots accumulating ∂L/∂x and ∂L/∂res (gxb, grb; -1: the
    // arena), gxf / grf = 1 on a tensor's first contribution (a store, not an
    // add); bsync as fsync, for the backward
    int gyb, gxb, grb, gxf, grf, bsync;
};

struct RbpParams {
    int B, K, A, H, P, Wb, obs_feat, arena, n_app, n_head, obs_t, intermediate_rewards, nflat, dt_floats;
    int xs_floats;                        // LDS: DT [dt_floats], XS [xs_floats], then the ring [.][dt_floats]
    const int2* gzero; int n_gzero;       // arena ∂L/∂t ranges {offset, floats} zeroed first (not ring-resident)
    const RbpApp* apps; const BpHead* heads;
    float* act; float* grad;              // [B][arena] activations / their gradients
    // LDS: [dt_floats] the application's ∂L/∂t, then its input (the largest conv input)
    const float* flat;
    const float* obs; const float* actions; const float* tv; const float* tr; const float* tp;
    const float* gscale; const float* weights;
    float* terms; float* pv; float* pp; float* pr;
    unsigned long long* stamps;           // diagnostic build (-DMZ_STAMPS) only: application end cycles of sample 0
};

// One layer of the ResNet nets (conv or dense) and its applications in the unroll
struct RbpLayer {
    int conv;                   // 1 conv, 0 dense
    int w_off, b_off, bn_off, cin, cout, kw, kh, act;
    int use0, n_use;            // uses[use0 .. use0 + n_use)
};
struct RbpUse { int x, y, z; }; // arena offsets of one application: input, output, pre-BatchNorm t
struct RbpJob { int layer, ob, kb; };   // a 16x16 block of dW; kb = -1: db (dβ, dγ) of channels ob·16 ..

#define RBP_DW_WAVES 4                    // mz_rbp_dw: waves per job
struct RbpDwParams {
    int B, P, Wb, arena;
    const RbpJob* jobs; const RbpLayer* layers; const RbpUse* uses;
    const float* act; const float* grad; const float* flat;
    float* out;                           // Flux-order data term of the gradient (2θ: mz_adam_kernel)
    double* sq;                           // [jobs]: Σθ² of each job's parameter block (f64, fixed order)
};
