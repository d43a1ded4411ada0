// mz_small_params.h — parameters and constants of the small-batch search
// kernel (mz_small.hip), shared with the host schedule builder.
#pragma once
#include "mz_internal.h"
#include "mz_selfplay_params.h"

// SM_SLOTS 64-row slots per stage, 256 threads each (build-time choice: more
// slots = fewer, wider stages and fewer resident weight registers per thread)
#ifndef SM_SLOTS
#define SM_SLOTS 2
#endif
#define SM_THREADS (256 * SM_SLOTS)
#ifndef SM_MAX_SIM
#define SM_MAX_SIM 8       // stages of the prediction ‖ dynamics schedule
#endif
#define SM_MAX_ROOT 6      // stages of the representation schedule

typedef float sm_f32x4 __attribute__((ext_vector_type(4)));

// Register image of one stage: [slot][chunk c = j/4][thread t of the slot][4],
// t = (slot row / 16)*64 + q*16 + slot row % 16 — thread (tid & 255) of the
// slot holds weight j of its (row, quarter) at chunk j/4, so every one of a
// wave's four float4 loads per stage reads 1 KiB contiguous (whole cache
// lines) instead of 16 B at a 64-B stride.
__host__ __device__ __forceinline__ size_t sm_widx(int stage, int slot, int q, int srow, int j) {
    const int t = (srow >> 4) * 64 + q * 16 + (srow & 15);
    return ((((size_t)stage * SM_SLOTS + slot) * 4 + (j >> 2)) * 256 + t) * 4 + (j & 3);
}

// Per wave of the workgroup (slot * 4 + 16-row group) and image stage (sim
// stages, then root stages), bit q*4 + c: chunk c (weights 4c..4c+3) of DPP
// row q holds a nonzero gather for some row of the group.  Chunks whose bit
// is clear are all zero in the image (an empty slot, a quarter past K, steps
// past kq): sm_load skips them.  [wave][stage], so a wave's masks are one
// scalar load.
#define SM_NZM_ST (SM_MAX_SIM + SM_MAX_ROOT)
#define SM_NZM_N (SM_NZM_ST * SM_SLOTS * 4)
// the array as passed: sm_load preloads a wave's SM_MAX_SIM masks in one
// batch of scalar loads from base + n_sim (root stages), whatever [k0, k1)
// it then uses, so the last wave's batch may reach SM_MAX_SIM - 1 entries past
// SM_NZM_N; the padding keeps that read inside the kernel-argument struct
#define SM_NZM_ALLOC (SM_NZM_N + SM_MAX_SIM)

// Per stage, the host-built record: one int4 per [slot][row] (copied to LDS)
//   .x  input base of the row's layer in the activation buffer (0 if unused:
//       the row's weights are zero and its output is dropped)
//   .y  kq of the layer (k steps per quarter)
//   .z  output offset of the row | relu << 30 | BatchNorm << 29, or -1 = unused row
//   .w  bias bits (filled at kernel start from the re-gathered bias image)
#define SM_REC_INTS (SM_SLOTS * 64 * 4)

struct SmallParams {
    int G, S, A, H, players, obs_feat, plane, exploration;
    uint32_t rng_step, game_offset;
    uint64_t seed;
    float temperature, discount, dirichlet_alpha, exploration_eps;
    const float* temp_g;   // per-game temperatures (self-play temperature_threshold) or NULL
    const float* obs; const uint8_t* legal; const int32_t* to_play;
    float* child_visits; float* root_value; int32_t* action_out;
    int n_sim, n_root;
    const float* w_sim;    // [n_sim] stage images (sm_widx)
    const float* w_root;   // [n_root] stage images (sm_widx)
    const int* rec;        // [n_sim + n_root][SM_REC_INTS] (bias slots filled from `bias`)
    const float* bias;     // [n_sim + n_root][slot][64] (re-gathered from the parameters)
    int act_total;
    int x_rep, x_pred, x_dyn, h_out, v_out, p_out, r_out;
    int v_act, r_act;
    const double* pbc_tab; const double* sqrt_tab; const float* aval_tab;
    const double* pbterm;  // pb_term triangle (mz_tree_device.h), copied to LDS
    char* tree; size_t tree_game_bytes; int dump_tree;
    unsigned long long* stamps;
    const float4* zero16;    // 16 zero bytes: the address of a skipped chunk's load
    uint32_t nzm[SM_NZM_ALLOC];  // nonzero-chunk masks [wave][stage]: sim stages, then root stages (+ pad)
    int bn;                  // BatchNorm FC layers: `bias` has γ and β sections after the biases
};

// Learner unroll on the small-kernel schedule (mz_unroll_small*): T samples
// per workgroup, the search's register images (kept current by ADAM).
struct SmallUnrollParams {
    int B, K, A, H, plane, obs_feat;
    const float* obs;      // (obs_feat, B)
    const float* actions;  // (K+1, B) float action ids
    float* pv; float* pp; float* pr;   // (K+1,B), (A,K+1,B), (K+1,B)
    int n_sim, n_root;
    const float* w_sim;    // [n_sim] stage images (sm_widx), as the search
    const float* w_root;   // [n_root] stage images (sm_widx)
    const float* bias;     // [n_sim + n_root][slot][64]
    const int* rec;        // [n_sim + n_root][SM_REC_INTS]
    int act_total;
    int x_rep, x_pred, x_dyn, h_out, v_out, p_out, r_out;
    int v_act, r_act;
    unsigned long long* stamps;   // -DMZ_STAMPS builds: [blocks][8] phase ticks (else unused)
    // fused get_batch (mz_learner_*_sampled): wave w < T of the workgroup first
    // draws sample tile0 + w from the replay shard into rp's batch arrays (obs
    // and actions are the arrays above), under the weight-image loads
    int sample;
    RpSampleParams rp;
    // get_batch prefetched by the previous launch (mz_engine.hip, learner_sampled):
    // this batch set's header {epoch, games played, step, B}; when it matches
    // (pf_epoch, rp.counters[0], rp.step, B) the set already holds this step's
    // batch and the sampling above is skipped.  nullptr: no prefetch.
    const long long* pf_hdr;
    long long pf_epoch;
    const float4* zero16;    // as SmallParams
    uint32_t nzm[SM_NZM_ALLOC];  // nonzero-chunk masks (as SmallParams)
    int bn;                  // as SmallParams
};

// One-launch learner step (mz_learn_small*, mz_learner_train_dev on one GPU,
// PER off): blocks [0, nU) are the unroll workgroups of SmallUnrollParams,
// which then compute their samples' loss terms; blocks [nU, nU + 48) run the
// Σθ² slices with ADAM (two 256-thread slices each) writing the new values into
// the engine's second image set, so the unroll blocks' weight loads never
// race them; the last block folds the losses.
struct LearnParams {
    int nU;
    int xcd;              // the unroll workgroups on physical blocks 0, 8, .. (grid 8·nU; learn_body)
    const float* tv; const float* tp; const float* gscale;
    float* terms; float* flat; const size_t* netoff; double* part; unsigned* counter; float* out;
    LgAdam ad;
    // blocks [nU + LEARN_L2_GROUPS, + pf_nb): get_batch of the next step (pfq:
    // the other batch set, step + 1), one wave per sample; the first of them
    // stamps pf_hdr_next
    int pf_nb;
    RpSampleParams pfq;
    long long* pf_hdr_next;
    long long pf_epoch;
};
// L consecutive ref_semantics learner steps t .. t+L-1 (mz_learner_train_multi_dev).
// Q11: the update θ_{s+1} = ADAM(θ_s, ∇ = 2θ_s) is elementwise and does not
// read the data, and with PER off step s's batch is keyed by s alone, so the L
// unrolls and losses are independent once θ_t .. θ_{t+L-1} exist.  Two launches:
//  * mz_learn_chain (256 threads): blocks [0, 3·MZ_L2_BLOCKS) run the L ADAM
//    iterations of their Σθ² slice in registers — Σθ_{t+i}² of the slice per i
//    (lg_l2_slice's order), θ_{t+i} scattered into bank image i, θ_{t+L} into
//    flat / M / V and the engine's current images;
//  * mz_learn_multi{1,2} (SM_THREADS): the L·⌈B/T⌉ unroll workgroups, each on
//    its step's bank image: waves 0..T-1 first draw the workgroup's samples of
//    step t+i (get_batch keyed by the step, one wave per sample), then the
//    unroll and the loss terms; the last workgroup of step i folds step i's
//    losses with the chain launch's Σθ² partials.  (MZ_MULTI_CHAIN_SAMPLE=1:
//    the chain launch draws the L batches in blocks after its slices instead.)
#define MZ_MULTI_MAX 32           // steps per chain launch (a bank half holds their images)
#define MZ_MULTI_UNROLL 16        // steps per unroll launch (FC: one workgroup per CU at B = 32, T = 2)
#define MZ_MULTI_LMAX 256         // steps per mz_learner_train_multi_dev call
#define MZ_MULTI_CNT_STRIDE 32   // per-step fold counters on their own 128-byte lines
struct ChainParams {
    int L;
    float* flat; float* M; float* V; const size_t* netoff;
    const int* inv_tile; const int* inv_small;
    float* Wp; float* Bp; float* smw; float* smb;     // the current images: θ_{t+L}
    float* bank_w; float* bank_b; size_t bws, bbs;     // bank image i (small-kernel W, bias): θ_{t+i} (or NULL)
    float* tbank_w; float* tbank_b; size_t tws, tbs;   // bank image i of the tile / ResNet MFMA image (or NULL)
    float* fbank;                                      // NULL or [L][fstride]: θ_{t+i}, the flat parameters of step t+i
    size_t fstride;                                    // nflat rounded up to 4 (16-byte rows: the downsampler's float4 reads)
    float* theta;                                      // NULL or [L][nflat]: θ after step t+i
    int cap_i[2]; float* cap_dst[2];                   // θ after step t+cap_i[j] -> cap_dst[j] (cap_i < 0: none;
                                                       // mz_train_run's actor / queued sets at refresh steps)
    float* cap_img[4];                                 // NULL or cap 0's search images (Wp, Bp, smw, smb): θ after
                                                       // step t+cap_i[0] scattered as into the engine's images
    size_t nflat;
    double* part;                                      // [L][3·MZ_L2_BLOCKS] Σθ_{t+i}² partials
    double bp1[MZ_MULTI_MAX], bp2[MZ_MULTI_MAX], eta[MZ_MULTI_MAX];   // step t+i's β powers, learning rate
    int B;                                             // batches: sample q = i·B + b, one wave each
    RpSampleParams q;                                  // step t's get_batch; step i's arrays at + i·stride
    size_t s_obs, s_k1, s_tp;                          // per-step strides: B·F, B·(K+1), B·(K+1)·A
    // helper workgroups (blocks [0, nh[0] + nh[1] + nh[2]), before the slices): net n's parameters past
    // the slices' first pass (e >= MZ_L2_BLOCKS·MZ_THREADS), one per thread, so no thread runs two
    // parameters' chains in sequence.  Every block of a slot with helpers stores its θ_{t+i} to
    // hx[i·hx_n + hoff[n] + e] (agent scope) and counts itself in at hcnt[n·MZ_L2_BLOCKS + slot]; the
    // last one adds the squares in lg_l2_slice's order (nh[n] = 0: the slice runs them itself)
    int nh[3];
    size_t hoff[3], hx_n;
    float* hx;
    unsigned long long* hcnt;                          // [3·MZ_L2_BLOCKS], a multiple of npart between launches
};
struct LearnMultiParams {
    int L, nU, xcd;                                    // xcd: step i on XCD i mod 8 (learn_multi_body)
    const float* bank_w; const float* bank_b; size_t bws, bbs;
    size_t s_obs, s_k1, s_tp;                          // as ChainParams (batch, read-outs, policies)
    const float* obs; const float* act; const float* tv; const float* tp; const float* gs;
    float* pv; float* pp; float* pr; float* terms;     // terms: [L][2·B·(K+1)]
    const double* part; unsigned* counter; float* out; // [L][3·MZ_L2_BLOCKS], [L][MZ_MULTI_CNT_STRIDE], [L][8]
    float* out_last;                                   // non-NULL: step L-1's losses go here instead (mz_train_run)
    int sample;                                        // waves 0..T-1 draw their samples (else mz_learn_chain did)
    RpSampleParams q;                                  // as ChainParams::q
};

// The loss terms and per-step folds of a multi-step sub-chunk whose unrolls
// ran in other launches (the ResNet nets, mz_learner_loss_multi): grid (nlb,
// L), step z = blockIdx.y on its arrays at + z·strides, the chain launch's
// Σθ² partials of the step, one fold counter per step.
struct LossMultiParams {
    int B, K, A, v_act, r_act, nlb, L;
    size_t s_k1, s_tp;
    float* pv; float* pp; float* pr; const float* tv; const float* tp; const float* gs; float* terms;
    const double* part; unsigned* counter; float* out; float* out_last;
};

// Σθ² / ADAM workgroups of the fused learner: 48 (each 256-thread half takes
// every 96th of the 3·MZ_L2_BLOCKS slices in turn; measured: one slice per
// half, 192 workgroups at 128 slices, ran 33.3 k vs 34.5 k steps/s at 48)
#define LEARN_L2_GROUPS 48
#define LEARN_L2_PASSES ((3 * MZ_L2_BLOCKS + LEARN_L2_GROUPS * SM_SLOTS - 1) / (LEARN_L2_GROUPS * SM_SLOTS))

