// mz_small_params.h — parameters and constants of the small-batch search
// kernel (mz_small.hip), shared with the host schedule builder.
#pragma once
#include "mz_internal.h"

#define SM_THREADS 256
#define SM_SLOTS 2
#define SM_MAX_SIM 8       // stages of the prediction ‖ dynamics schedule
#define SM_MAX_ROOT 6      // stages of the representation schedule

typedef float sm_f32x4 __attribute__((ext_vector_type(4)));

// Per stage, the host-built record (ints, copied to LDS):
//   [0..1]      kq of slot 0 / 1 (k steps per quarter; 0 = slot idle)
//   [2..129]    xb[slot][lane]: B-operand base = in_off + (lane & 3), -1 = zero
//   [130..257]  ob[slot][row]: output offset of slot row r (-1 = unused)
//   [258..385]  bias bits [slot][row]
//   [386..513]  relu flag [slot][row]
#define SM_REC_INTS (2 + 4 * 128)

struct SmallParams {
    int G, S, A, H, players, obs_feat, plane, exploration;
    uint32_t rng_step, game_offset;
    uint64_t seed;
    float temperature, discount, dirichlet_alpha, exploration_eps;
    const float* obs; const uint8_t* legal; const int32_t* to_play;
    float* child_visits; float* root_value; int32_t* action_out;
    int n_sim, n_root;
    const float* w_sim;    // [n_sim][slot][q*64 + lane][16]
    const float* w_root;   // [n_root][slot][q*64 + lane][16]
    const int* rec;        // [n_sim + n_root][SM_REC_INTS] (bias slots filled from `bias`)
    const float* bias;     // [n_sim + n_root][slot][64] (re-gathered from the parameters)
    int act_total;
    int x_rep, x_pred, x_dyn, h_out, v_out, p_out, r_out;
    int v_act, r_act;
    const double* pbc_tab; const double* sqrt_tab; const float* aval_tab;
    char* tree; size_t tree_game_bytes; int dump_tree;
    unsigned long long* stamps;
};

