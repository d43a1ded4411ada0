// mz_resnet_params.h — plans of the ResNet networks (row a14) shared by the
// host plan builder (mz_engine.hip) and the kernels (mz_resnet.hip).
//
// Every op is a generalised Dense  y[o][n] = Σ_k W[o][k] · B(k, n)  on a tile
// of NG games.  Activations live in LDS as [feature][game] with feature
// f = p + P·c for a (W, H, C) conv tensor (p = w + W·h): a conv layer has
// P·NG columns n = p·NG + g, a Dense layer (after Flux.flatten, which is the
// same column-major order) has NG columns.  K order of a conv: k = i + kw·j +
// kw·kh·c (the Flux weight's column-major order); B(k, n) of a kernel > 1x1
// reads x[w + (kw-1-i) - pw, h + (kh-1-j) - ph, c] (Flux convolution, kernel
// flipped) or 0 outside the board.
#pragma once
#include "mz_selfplay_params.h"

#define RN_MAX_LAYERS 96
#ifndef RN_THREADS
#define RN_THREADS 512           // root / unroll / forward kernels: 8 waves, 2 per SIMD
#endif
#ifndef RN_THREADS_NETS
#define RN_THREADS_NETS 768      // search network launch: 12 waves, 3 per SIMD (one unit of a 64x144 conv each)
#endif

// Activation buffer layouts.  Plain: x[k][n] at k·ncols + n (k = feature /
// channel, n = column).  K-blocked (for readers whose MFMA B operands walk k in
// steps of 4: 1x1 convs and Dense layers with K % 64 == 0): with k = 4m + kl,
// element (k, n) sits at ((m >> 2)·ncols + n)·16 + 4·(((n >> 2) & 3) ^ σ(kl)) +
// (m & 3), σ = (0, 3, 1, 2), so the four k-steps 4M..4M+3 a lane (kl = lane >>
// 4, n = lane & 15) feeds to consecutive MFMAs are one 16-byte LDS read, and the
// σ swizzle keeps each ds_read_b128 lane group on distinct banks.
__host__ __device__ __forceinline__ int rn_kb_sigma(int kl) { return (0x2130 >> (4 * kl)) & 3; }
__host__ __device__ __forceinline__ int rn_kb_off(int k, int n, int ncols) {
    return ((k >> 4) * ncols + n) * 16 + 4 * (((n >> 2) & 3) ^ rn_kb_sigma(k & 3)) + ((k >> 2) & 3);
}

struct RLayer {
    int kk;              // kw * kh (1: Dense or 1x1 conv; > 1: im2col gather through the k table)
    int kw, kh, pw, ph;
    int K, cout;         // reduction length, output rows (channels / features)
    int nq, n_ob;        // k-steps per quarter (ceil(K/16)), 16-row output blocks
    int spatial;         // columns = P·NG (conv) or NG (Dense)
    int act, bn, res_add;
    int w_img;           // packed A fragments [n_ob][4][nq4/4][64][4] in the image (nq4 = 4⌈nq/4⌉)
    int boff, bnoff;     // absolute offsets in the flat parameters (bias; β then γ)
    int in_off, out_off, res_off;   // LDS offsets (floats)
    int ktab;            // LDS offset of the k table (kk > 1), else -1
    int in_kb, out_kb, res_kb;   // input / output / residual buffer in the k-blocked layout (rn_kb_off)
    int ep_img;          // epilogue image [n_ob·16 rows][bias, γ, β, 0] in the weight image (after the A fragments)
    int otab;            // kernel > 1x1 read through a per-lane offset table at LDS int offset ktab (narrow plans)
};

// What the layer loop reads per layer, packed into 8 words so a layer's entry
// is one scalar load (rn_rk_decode): flags, K | cout, nq | n_ob, in | out, res |
// ktab (16-bit LDS offsets), w_img, ep_img
struct RK { int w[8]; };
enum { RK_KK = 1, RK_SPATIAL = 2, RK_BN = 16, RK_RES = 32, RK_IN_KB = 64, RK_OUT_KB = 128, RK_RES_KB = 256,
       RK_OTAB = 512 };
__host__ __device__ __forceinline__ RK rn_rk_pack(const RLayer& L) {
    RK k;
    k.w[0] = (L.kk > 1 ? RK_KK : 0) | (L.spatial ? RK_SPATIAL : 0) | (L.act << 2) | (L.bn ? RK_BN : 0) |
             (L.res_add ? RK_RES : 0) | (L.in_kb ? RK_IN_KB : 0) | (L.out_kb ? RK_OUT_KB : 0) |
             (L.res_kb ? RK_RES_KB : 0) | (L.otab ? RK_OTAB : 0);
    k.w[1] = L.K | (L.cout << 16);
    k.w[2] = L.nq | (L.n_ob << 16);
    k.w[3] = L.in_off | (L.out_off << 16);
    k.w[4] = (L.res_off & 0xffff) | (L.ktab << 16);
    k.w[5] = L.w_img;
    k.w[6] = L.ep_img;
    k.w[7] = 0;
    return k;
}
// the fields rn_layer_t reads (kk only as "> 1"; kw/kh/pw/ph, boff/bnoff unused there)
__host__ __device__ __forceinline__ RLayer rn_rk_decode(const RK& k) {
    RLayer L;
    L.kk = (k.w[0] & RK_KK) ? 2 : 1; L.kw = L.kh = L.pw = L.ph = 0;
    L.spatial = (k.w[0] & RK_SPATIAL) != 0; L.act = (k.w[0] >> 2) & 3; L.bn = (k.w[0] & RK_BN) != 0;
    L.res_add = (k.w[0] & RK_RES) != 0; L.in_kb = (k.w[0] & RK_IN_KB) != 0; L.out_kb = (k.w[0] & RK_OUT_KB) != 0;
    L.res_kb = (k.w[0] & RK_RES_KB) != 0; L.otab = (k.w[0] & RK_OTAB) != 0;
    L.K = k.w[1] & 0xffff; L.cout = (int)((unsigned)k.w[1] >> 16);
    L.nq = k.w[2] & 0xffff; L.n_ob = (int)((unsigned)k.w[2] >> 16);
    L.in_off = k.w[3] & 0xffff; L.out_off = (int)((unsigned)k.w[3] >> 16);
    L.res_off = k.w[4] & 0xffff; L.ktab = k.w[4] >> 16;
    L.w_img = k.w[5]; L.ep_img = k.w[6];
    L.boff = L.bnoff = 0;
    return L;
}

struct RPlan {
    int n;
    RLayer L[RN_MAX_LAYERS];
    RK k[RN_MAX_LAYERS];               // the same layers packed (rn_rk_pack)
    int in_off, in_feat;               // input buffer (features x NG)
    int in_kb;                         // the staged input is k-blocked (its first readers are 1x1 / Dense, K % 64 == 0)
    int out0_off, out0_n;              // out0: h (REPR, DYN) or value (PRED)
    int out0_kb;                       // out0 k-blocked (h of the dynamics, when its state head reads it so)
    int out1_off, out1_n;              // out1: policy logits (PRED) or reward (DYN), n = 0 if none
    int out0_act, out1_act;            // the activation of the layer writing out0 / out1 (rn_run<.., RAWTANH>
                                       // leaves a tanh unapplied in LDS; the caller applies it on read-out)
    int lds_floats;                    // LDS per workgroup (floats), k tables included
    // narrow (learner chain) plans: the B-operand byte offsets of the layers with a
    // kernel > 1x1 ([q][chunk][column][slot][4 k-steps], rn_otab_fill), copied
    // from the engine's table buffer at tab_src to LDS at tab_lds (tab_n ints) by
    // the kernel; zero_off = an LDS float kept 0 (out-of-board taps, padding)
    int tab_src, tab_lds, tab_n, zero_off;
    int n_ktab;                        // layers with a k table (kernel > 1x1 read through rn_fill_ktabs' tables)
};

struct RNetParams {
    int ng, W, H, P;                   // tile width, board
    int n_items;                       // items (games / samples) in total
    int softmax1;                      // out1 is a policy: write probabilities (mz_net_forward)
    float bn_s;                        // sqrtf(1 + 1e-5): BatchNorm test-mode denominator (σ² = 1)
    const RPlan* plan;                 // device copy
    const float* Wimg;                 // packed A fragments
    const float* flat;                 // Flux-order parameters (biases, BatchNorm)
    const float* x;                    // (in_feat, n_items) column-major input
    float* out0; float* out1;          // (out0_n, n_items), (out1_n, n_items)
};

// Batched search with the ResNet networks: a root launch, then per
// simulation a tree step (16 lanes per game; trees and hidden states in HBM)
// and one network launch (prediction ‖ dynamics).  Per-game state gst[g][16]:
// legal, root_tp, rootN, rootW, mmin, mmax, leaf_e, leaf_a, vtp, depth.
enum { RG_LEGAL = 0, RG_ROOT_TP, RG_ROOTN, RG_ROOTW, RG_MMIN, RG_MMAX, RG_LEAF_E, RG_LEAF_A, RG_VTP, RG_DEPTH,
       RG_VER,                          // the LDS tree step's cached-select tag (mz_tree_device.h select_path_cached)
       RG_XK,                           // doublings of the leaf_e node's h before this simulation (RSearchParams::hk)
       RG_INTS = 16 };

struct RSearchParams {
    int G, S, A, H, W, P, players, obs_feat, exploration, s;
    uint32_t rng_step, game_offset;
    uint64_t seed;
    float temperature, discount, dirichlet_alpha, exploration_eps;
    const float* temp_g;   // per-game temperatures (self-play temperature_threshold) or NULL
    const float* obs; const uint8_t* legal; const int32_t* to_play;
    float* child_visits; float* root_value; int32_t* action_out;
    const double* pbc_tab; const double* sqrt_tab; const float* aval_tab;
    const double* pbterm;  // the pb_term triangle (mz_tree_device.h pbterm_index), the recompute's table
    char* tree; size_t tree_game_bytes;
    float* hid;            // [G][S+1][H]
    uint2* cache;          // [G][S+1] the LDS tree step's cached select entries, home between launches
    int* nN;               // [G][S+1] N of each expanded node (the edge into it; the root's N), for recomputes
    int* path;             // [G][2(S+2)]
    int* gst;              // [G][RG_INTS]
    // make_state_action (Q1) doubles the parent's stored h in place at every use; a node's stored h is its
    // h' times 2^hk (hk = its uses so far, exact: powers of two), so the tree step only counts the use
    // (gst[RG_XK] = hk before it, then hk + 1) and the network launch reads hid[leaf_e] scaled by 2^hk
    // (prediction) and 2^(hk+1) (dynamics) — no copy of h, no rewrite of hid
    int* hk;               // [G][S+1]
    float* o_v; float* o_logit; float* o_r;   // [G], [G][A], [G]
    int ng; float bn_s;
    const RPlan* plans;    // repr, pred, dyn
    unsigned long long* stamps;   // -DMZ_STAMPS builds: per-layer ticks of nets blocks (0,0), (0,1)
    const float* Wimg; const float* flat;
    // rew_split (mz_rsearch_nets): y = 0 runs the dynamics trunk, publishes its
    // output (trunk[G][H], agent-scope stores, then tprog[tile] = tepoch) and runs
    // the state head; y = 1 runs the prediction, then the dynamics reward head
    // ([dyn_split, n)) on the published trunk output — the two workgroups of a
    // tile carry about equal work instead of 101 k / 142 k ticks
    int rew_split, trunk_nl, dyn_split;
    float* trunk; unsigned long long* tprog; unsigned long long tepoch;
    unsigned* fault;                   // MZ_FAULT_RS_TRUNK on a publish that never came (mz_poll_ge)
    unsigned long long poll_ticks;     // the poll's bound (MZ_POLL_TICKS)
    int dbg_skip;                      // debug: the tile whose trunk publish is skipped (-1 = none)
    int no_moved_skip;                 // A/B only (MZ_NO_MOVED_SKIP): after a min / max move the walk starts at the root
};

// LDS layout of the LDS-cached tree step (mz_rsearch_tree_lds*): one wave per
// workgroup, 64/GW games.  Shared: the pUCT tables pbc[S+2], sqrt[S+2] (f64).
// Per game: the tree copy (tree_game_bytes, +16 for the dword copy of the
// to_play bytes), the path [2(S+2)] ints, rr / vin [S+2] floats (1-player
// backup), the GW-float softmax staging slot.
#ifndef RT_WAVES
#define RT_WAVES 8                     // waves of the LDS-cached tree step (mz_rsearch_tree_lds*)
#endif
struct RsTreeLds { int tables, game, tree, path, rr, vin, stg, cache, lvl, nn, total; };
__host__ __device__ __forceinline__ int rs_align16(size_t x) { return (int)((x + 15) & ~(size_t)15); }
__host__ __device__ __forceinline__ RsTreeLds rs_tree_lds(int S, size_t tree_game_bytes, int GW) {
    RsTreeLds L;
    L.tables = rs_align16((size_t)16 * (S + 2));
    L.tree = 0;
    L.path = rs_align16(tree_game_bytes + 16);
    L.rr = L.path + rs_align16((size_t)8 * (S + 2));
    L.vin = L.rr + rs_align16((size_t)4 * (S + 2));
    L.stg = L.vin + rs_align16((size_t)4 * (S + 2));
    L.cache = L.stg + rs_align16((size_t)4 * GW);           // uint2 [S+1] entries
    L.lvl = L.cache + rs_align16((size_t)8 * (S + 1));      // uint2 [S+2] (slot, N) per path level (backup)
    L.nn = L.lvl + rs_align16((size_t)8 * (S + 2));         // int [S+1] N per expanded node
    L.game = L.nn + rs_align16((size_t)4 * (S + 1));
    L.total = L.tables + (64 / GW) * L.game;
    return L;
}

// Learner unroll with the ResNet networks (Learning.jl:347-370, Q10): per
// tile of NG samples, representation, then K x (prediction(h), dynamics(2h ⊕
// a/|A|)); h is handed between the nets through hs.  Raw outputs as the FC
// unroll: value / reward already activated, policy logits.
struct RUnrollParams {
    int B, K, A, H, W, P, obs_feat, ng;
    float bn_s;
    const float* obs; const float* actions;
    float* pv; float* pp; float* pr;   // (K+1, B), (A, K+1, B), (K+1, B)
    float* hs;                         // [B][H] scratch (mz_runroll_kernel); [B][K][H] h_0..h_{K-1} (split form)
    const RPlan* plans;
    const float* Wimg; const float* flat;
    // split form: mz_runroll_chain (representation + the K dynamics steps, the
    // sequential part) on tiles of ng_l samples with plans_l, then
    // mz_runroll_pred (the K predictions, independent) on tiles of ng items
    const RPlan* plans_l; int ng_l;
    const int* otab;                   // the narrow plans' offset tables (RPlan.tab_src)
    int dyn_split;                     // first reward-head layer of the dynamics plans
    float* ts;                         // [B][K][H] dynamics trunk outputs (split form: the reward heads' input)
    unsigned long long* stamps;        // -DMZ_STAMPS builds: per-layer ticks of chain block 0 (repr, dyn s = 1)
    int rd_ep_off;                     // mz_runroll_chain_r: LDS float offset of the staged epilogue parameters
    int rd_trunk_nl;                   // mz_runroll_chain_r: the dynamics trunk's layers (1 + 2·num_blocks); the
                                       // last step runs only these (its h_K feeds nothing in the unroll)
    // mz_runroll_fused_r (one launch: chain blocks [0, n_chain), then the B·K
    // prediction / reward-head items, each waiting for its sample's chain):
    // prog[b] = prog_base + p once the chain of sample b has stored h_0..h_{p-1}
    // and the trunk outputs of steps 1..p-1 (prog_base = launch epoch · 64)
    unsigned long long* prog; unsigned long long prog_base;
    int n_chain;
    int fuse_sample;                   // 1: chain block b draws sample b (get_batch, rq) first
    RpSampleParams rq;
    // n_l2 > 0 (one GPU, ADAM fused): blocks [n_chain, n_chain + n_l2) take the
    // Σθ² slices of mz_learner_grad_kernel (lg_l2_slice: Σθ² into part, ADAM on
    // flat_w in place, the new MFMA image into ad.Wp = the second image set,
    // which the kernels of this launch do not read); the loss kernel then runs
    // without its slice blocks
    int n_l2;
    LgAdam ad; float* flat_w; const size_t* netoff; double* part;
    int rp_nv;                         // the prediction plan's value-head layers ([RP_NL, RP_NL + rp_nv)); the
                                       // fused launch runs the value and the policy head of an item in two blocks
    unsigned* fault;                   // MZ_FAULT_RD_PROGRESS on a publish that never came (mz_poll_ge)
    unsigned long long poll_ticks;     // the poll's bound (MZ_POLL_TICKS)
    int dbg_skip;                      // debug: the chain block (sample) whose publishes are skipped (-1 = none)
    // ms > 0: a multi-step launch (mz_learner_train_multi_dev, ref_semantics): blockIdx.z = step z of the
    // sub-chunk, which reads its own parameters (Wimg + z·ms_wimg, flat + z·ms_flat) and batch (obs,
    // actions, rq at + z·strides), writes its read-outs and scratch at + z·strides and publishes / polls its
    // own progress words (prog + z·B); rq.step + z keys its get_batch (rn_step)
    int ms;
    size_t ms_wimg, ms_flat, ms_obs, ms_k1, ms_tp, ms_hs;
};
// mz_runroll_chain_r: the dynamics chain's layers ([0, dyn_split) = RD_NL:
// trunk + state head of 2-block towers) with register-resident A fragments
#define RD_NL 10
#define RD_NL3 18        // mz_runroll_chain_r3: 4-block towers on three column blocks (Connect4 ResNet-8)
#define RD_THREADS 256
// mz_runroll_pred_r: the prediction trunk's RP_NL layers (1 + 2 blocks) the same way
#define RP_NL 5

// Downsampler of the ResNet representation (ResNetHP.downsample,
// Learning.jl:175-187; BASELINE configs[4]): stride-2 convs without
// BatchNorm, residual blocks and MeanPool((3,3), stride 2, pad 1) taking the
// (84, 84, C) observation to (6, 6, 2C), which the representation's tail
// (conv 2C -> nf + blocks, an RPlan) reads.  One workgroup per item; the
// activations ping-pong between two LDS buffers [c][h][w] (the column-major
// (W, H, C) order); the observation is staged in LDS for the first layer.
#define DS_MAX_LAYERS 32
#define DS_THREADS 512
enum { DS_CONV = 0, DS_POOL = 1 };
struct DsLayer {
    int kind, cin, cout, kw, kh, pw, ph, stride;
    int Wi, Hi, Wo, Ho;
    int act, bn, res_add;
    int woff, boff, bnoff;   // absolute offsets in the flat parameters (conv)
    int in_buf, out_buf;     // LDS buffer 0 / 1, or -1 = the observation (in) / the output (out)
    int res_buf;             // residual buffer (res_add)
    int pn;                  // conv: its parameters W, b (, β, γ) contiguous from woff (pn floats); pool: 0
};
struct DsPlan {
    int n;
    DsLayer L[DS_MAX_LAYERS];
    int buf_floats;          // floats per activation buffer
    int w_floats;            // largest conv weight block (K x cout)
    int in_feat, out_feat;   // W*H*C of the observation / of the output
    // mz_downsample_kernel's LDS beyond the two buffers: the observation staged
    // for layer 0 (stage_in: from buf_floats, where buffer 1 starts, over
    // in_feat floats); after layer 0 every conv's parameters (W, b, β, γ,
    // contiguous from L[0].woff over ptot floats) at 2·buf_floats, inside the
    // staging region; layer 0's own at lds_floats (pn_max floats)
    int stage_in, pn_max, ptot;
    int lds_floats;          // buffers + staging region
};
struct DsParams {
    int n_items;
    float bn_s;
    const DsPlan* plan;
    const float* flat;
    const float* x;          // (in_feat, n_items) column-major
    float* y;                // (out_feat, n_items)
    unsigned long long* stamps;   // -DMZ_STAMPS builds: item 0's s_memtime at each layer's end (else unused)
    int per_step;            // > 0 (multi-step learner): item i uses the parameters flat + (i / per_step)·flat_stride
    size_t flat_stride;
};

// ---- the corrected learner through the downsampler (mz_dsbp_*, mz_downsample.hip)
// Per-sample arenas in HBM hold every downsampler layer's output y (the column-
// major (W, H, C) order) and, for BatchNorm convs, t = W x + b; the gradient
// arena the same tensors' ∂L/∂y.  The last layer's ∂L/∂y is the ResNet
// corrected learner's ∂L/∂(representation input) (mz_rbp_sample).
struct DsBpLayer { int x, y, z, res; };   // arena offsets: input (-1: the observation), output, t (-1), residual
struct DsBpParams {
    int B, arena;
    float bn_s;
    const DsPlan* plan; const DsBpLayer* lay;
    const float* flat;
    const float* obs;                     // (in_feat, B)
    float* act; float* grad;              // [B][arena]
    float* out;                           // forward: the downsampler output (out_feat, B)
    const float* gout; int gstride, goff; // backward: ∂L/∂output of sample b at gout[b·gstride + goff + f]
    int dt_off;                           // backward: the current conv's ∂L/∂t in the gradient arena
};
struct DsDwJob { int layer, co, ci; };    // one (output, input) channel pair of a conv: its taps; ci = 0 also b (β, γ)
#define DS_DW_THREADS 256
struct DsDwParams {
    int B, arena, n_job;
    float bn_s;
    const DsPlan* plan; const DsBpLayer* lay; const DsDwJob* jobs;
    const float* obs; const float* act; const float* grad; const float* flat;
    float* out;                           // Flux-order data term of the gradient
    double* sq;                           // [n_job]: Σθ² of each job's parameters
};
