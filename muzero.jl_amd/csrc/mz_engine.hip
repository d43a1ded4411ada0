// mz_engine.hip — host side of libmz: the C ABI of include/mz.h.
//
// Builds the layer/plan description of the FeedForwardHP networks
// (Learning.jl:87-142), packs Flux-order weights into the MFMA fragment
// image, owns every device buffer of one engine (one handle per GPU), and
// launches the search / forward / learner kernels on the handle's stream.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "mz_internal.h"
#include "mz_tree_device.h"   // tree_bytes (tree layout shared with the kernels)

static const size_t kLdsMax = 160 * 1024;   // LDS per workgroup on gfx950

extern "C" __global__ void mz_search_kernel_lds(SearchParams P);
extern "C" __global__ void mz_search_kernel_hbm(SearchParams P);
extern "C" __global__ void mz_search_kernel_lds_res(SearchParams P);
#include "mz_small_params.h"
#include "mz_resnet_params.h"
#include "mz_backprop_params.h"
#include "mz_selfplay_params.h"
#include "mz_ckpt_iface.h"
extern "C" __global__ void mz_rnet_forward_kernel(RNetParams Q);
extern "C" __global__ void mz_rsearch_root(RSearchParams P);
extern "C" __global__ void mz_rsearch_tree(RSearchParams P);
extern "C" __global__ void mz_rsearch_root32(RSearchParams P);
extern "C" __global__ void mz_downsample_kernel(DsParams Q);
extern "C" __global__ void mz_dsbp_fwd(DsBpParams Q);
extern "C" __global__ void mz_dsbp_bwd(DsBpParams Q);
extern "C" __global__ void mz_dsbp_dw(DsDwParams Q);
extern "C" __global__ void mz_rsearch_tree32(RSearchParams P);
extern "C" __global__ void mz_rsearch_tree_lds(RSearchParams P);
extern "C" __global__ void mz_rsearch_tree_lds32(RSearchParams P);
extern "C" __global__ void mz_rsearch_nets(RSearchParams P);
extern "C" __global__ void mz_runroll_kernel(RUnrollParams U);
extern "C" __global__ void mz_runroll_chain(RUnrollParams U);
extern "C" __global__ void mz_bp_tile(BpParams Q);
extern "C" __global__ void mz_bp_tile_lv(BpParams Q);
extern "C" __global__ void mz_bp_tile_lv_nobn(BpParams Q);
extern "C" __global__ void mz_bp_dw(BpDwParams Q);
extern "C" __global__ void mz_rbp_sample(RbpParams Q);
extern "C" __global__ void mz_rbp_dw(RbpDwParams Q);
extern "C" __global__ void mz_bp_fold(BpFoldParams Q);
extern "C" __global__ void mz_runroll_pred(RUnrollParams U);
extern "C" __global__ void mz_runroll_pred_n(RUnrollParams U);
extern "C" __global__ void mz_runroll_pred_n1(RUnrollParams U);
extern "C" __global__ void mz_runroll_chain1(RUnrollParams U);
extern "C" __global__ void mz_runroll_chain_r(RUnrollParams U);
extern "C" __global__ void mz_runroll_chain_r3(RUnrollParams U);
extern "C" __global__ void mz_runroll_pred_r(RUnrollParams U);
extern "C" __global__ void mz_runroll_fused_r(RUnrollParams U);
extern "C" __global__ void mz_runroll_fused_r3(RUnrollParams U);
extern "C" __global__ void mz_sp_prepare(SpParams S);
extern "C" __global__ void mz_sp_commit(SpParams S);
extern "C" __global__ void mz_sp_order(SpParams S);
extern "C" __global__ void mz_sp_store(SpParams S);
extern "C" __global__ void mz_sp_reset(SpParams S);
extern "C" __global__ void mz_rp_sample(RpSampleParams Q);
extern "C" __global__ void mz_rp_per_init(SpHist ring, int slot, int len, int Tmax, int td, const float* disc_pow,
                                          int alpha);
extern "C" __global__ void mz_rp_per_prep(SpHist ring, const long long* counters, int cap, float* cum, float* prob,
                                          long long* total);
extern "C" __global__ void mz_rp_per_norm(float* w, int B);
extern "C" __global__ void mz_rp_per_update(SpHist ring, const long long* counters, int cap, int Tmax, int B, int K,
                                            int alpha, const int32_t* index, const float* pv, const float* tv);
extern "C" __global__ void mz_search_small1(SmallParams P);
extern "C" __global__ void mz_search_small2(SmallParams P);
extern "C" __global__ void mz_search_small4(SmallParams P);
extern "C" __global__ void mz_search_small1_bn(SmallParams P);
extern "C" __global__ void mz_search_small2_bn(SmallParams P);
extern "C" __global__ void mz_search_small4_bn(SmallParams P);
extern "C" __global__ void mz_unroll_small1(SmallUnrollParams P);
extern "C" __global__ void mz_unroll_small2(SmallUnrollParams P);
extern "C" __global__ void mz_unroll_small1_bn(SmallUnrollParams P);
extern "C" __global__ void mz_unroll_small2_bn(SmallUnrollParams P);
extern "C" __global__ void mz_learn_small1(SmallUnrollParams P, LearnParams L);
extern "C" __global__ void mz_learn_small2(SmallUnrollParams P, LearnParams L);
extern "C" __global__ void mz_learn_small1_bn(SmallUnrollParams P, LearnParams L);
extern "C" __global__ void mz_learn_small2_bn(SmallUnrollParams P, LearnParams L);
extern "C" __global__ void mz_learn_chain(ChainParams C);
extern "C" __global__ void mz_learn_multi1(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learn_multi2(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learn_multi1_bn(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learn_multi4(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learn_multi4_bn(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learn_multi2_bn(SmallUnrollParams P, LearnMultiParams M);
extern "C" __global__ void mz_learner_loss_multi(LossMultiParams M);
extern "C" __global__ void mz_learner_loss_multi32(LossMultiParams M);
extern "C" __global__ void mz_search_kernel_hbm_res(SearchParams P);

extern "C" __global__ void mz_unroll_kernel(UnrollParams P);
extern "C" __global__ void mz_forward_kernel(const int* plan, const float* Wp, const float* Bp, int total_lds,
                                             int in_off, int in_feat, const float* x, int n, int out0_off, int o0,
                                             float* out0, int out1_off, int o1, float* out1, int sm1, int act0,
                                             int act1);
extern "C" __global__ void mz_learner_grad_kernel(int B, int K, int A, int v_act, int r_act, float* pv, float* pp,
                                                  float* pr, const float* tv, const float* tp, const float* gscale,
                                                  float* terms, float* flat, const size_t* netoff, float* G,
                                                  double* part, unsigned* counter, float* out, const float* wts, LgAdam ad);
extern "C" __global__ void mz_learner_grad_kernel32(int B, int K, int A, int v_act, int r_act, float* pv, float* pp,
                                                    float* pr, const float* tv, const float* tp, const float* gscale,
                                                    float* terms, float* flat, const size_t* netoff, float* G,
                                                    double* part, unsigned* counter, float* out, const float* wts, LgAdam ad);
extern "C" __global__ void mz_adam_kernel(float* P, float* M, float* V, const float* G, float gscale, size_t n,
                                          double bp1, double bp2, double eta, float* Wp, float* Bp,
                                          const int* inv_tile, float* smw, float* smb, const int* inv_small);
extern "C" __global__ void mz_repack_kernel(const float* flat, const int* src, float* packed, size_t n);

namespace {

enum { CH_TRUNK = 0, CH_HEAD1 = 1, CH_HEAD2 = 2 };

struct LayerSpec {
    int net, chain, in, out, act;
    size_t flux_w, flux_b;     // offsets in the global flat parameter vector
    int bn = 0;                // make_dense with use_batch_norm: BatchNorm β at flux_be, γ at flux_be + out
    size_t flux_be = 0;
    int nq, n_ob;
    int packed_w, packed_b;    // offsets in the packed images
};

struct PlanBuild {
    std::vector<std::vector<std::pair<int, int>>> stages;
    std::vector<LayerDesc> layers;
    void ensure(int n) { if ((int)stages.size() < n) stages.resize(n); }
    std::vector<int> image() const {
        std::vector<int> v;
        int nt = 0;
        for (auto& s : stages) nt += (int)s.size();
        v.push_back((int)stages.size()); v.push_back((int)layers.size()); v.push_back(nt);
        int acc = 0;
        for (auto& s : stages) { v.push_back(acc); acc += (int)s.size(); }
        v.push_back(acc);
        for (auto& s : stages) for (auto& t : s) { v.push_back(t.first); v.push_back(t.second); }
        for (auto& L : layers) {
            const int* p = reinterpret_cast<const int*>(&L);
            for (size_t i = 0; i < sizeof(LayerDesc) / sizeof(int); ++i) v.push_back(p[i]);
        }
        return v;
    }
};

thread_local std::string g_create_error;

}  // namespace

struct mz_handle {
    mz_config conf;
    mz_ffhp hp;
    int kind = 0;                           // 0 FeedForwardHP, 1 ResNetHP
    mz_resnet_hp rhp{};
    // ResNet config of the networks after the downsampler (= conf without
    // one): observation_shape = the representation tail's input board and
    // channels, stacked_observations = 0 (ResNetHP.downsample, configs[4])
    mz_config rconf{};
    int ds = 0;                             // downsampler (mz_downsample.hip) on
    DsPlan dsplan{};
    DsPlan* d_dsplan = nullptr;
    size_t ds_lds = 0, ds_n = 0;            // its LDS bytes, its parameter count (first in the repr net)
    int rin_feat = 0;                       // representation tail input features (obs_feat without downsampler)
    float* d_dsout = nullptr;               // [max_games][rin_feat] search roots' downsampled observations
    float* d_dsb = nullptr; int dsb_cap = 0;   // [cap][rin_feat] scratch: learner batches, net_forward
    // ResNet networks (mz_resnet.hip): host plans, device copies, tile width
    std::vector<RPlan> rplan;               // [3]
    RPlan* d_rplan = nullptr;               // [3]
    int rn_ng = 0;
    // the learner unroll's chain (mz_runroll_chain): the same nets on narrow tiles
    std::vector<RPlan> rplan_l;
    RPlan* d_rplan_l = nullptr;
    int rn_ng_l = 0;
    size_t rn_lds_l = 0;
    size_t rn_lds[3] = {0, 0, 0};
    float bn_s = 1.0f;
    int* d_rpath = nullptr; int* d_rgst = nullptr;          // ResNet search: [G][2(S+2)], [G][RG_INTS]
    uint2* d_rcache = nullptr; int* d_rnN = nullptr;        // [G][S+1]: the LDS tree step's cached select
    int* d_rhk = nullptr; float* d_rov = nullptr; float* d_rologit = nullptr; float* d_ror = nullptr;
    float* d_rhs = nullptr;                 // [bcap][K][H] learner unroll scratch (h between the nets)
    float* d_rts = nullptr;                 // [bcap][K][H] dynamics trunk outputs (the reward heads' input)
    int rn_dyn_split = 0;                   // first reward-head layer of the dynamics plan
    bool rd_chain = false;                  // the chain runs as mz_runroll_chain_r[3] (rd_chain_ok)
    int rd_nb = 1;                          // its column blocks (1: mz_runroll_chain_r, 3: _r3)
    bool rp_pred = false;                   // one-item predictions run as mz_runroll_pred_r (rp_pred_ok)
    unsigned long long* d_prog = nullptr;   // [bcap] mz_runroll_fused_r progress words
    float* d_rtrunk = nullptr;              // [max_games][H] dynamics trunk outputs (mz_rsearch_nets rew_split)
    unsigned long long* d_tprog = nullptr;  // [tiles] their publish words
    unsigned long long tprog_epoch = 0;     // mz_rsearch_nets launches
    float* d_chx = nullptr;                 // [MZ_MULTI_MAX][hx_n] mz_learn_chain helpers' θ (ChainParams::hx)
    unsigned long long* d_chcnt = nullptr;  // [3·MZ_L2_BLOCKS] their slots' arrival counters
    unsigned long long prog_epoch = 0;      // launches of mz_runroll_fused_r (prog_base = epoch · 64)
    std::vector<int> rtab;                  // offset tables of the narrow (chain) plans
    int* d_rtab = nullptr;
    int device = 0, max_games = 0;
    uint64_t seed = 0;
    std::string err;
    hipStream_t stream = nullptr;
    hipStream_t sync_stream = nullptr; bool sync_narrow = false;   // mz_set_sync_stream

    std::vector<LayerSpec> layers;
    std::vector<int> chains[3][3];          // [net][chain] -> layer indices
    size_t nparams[3] = {0, 0, 0}, flat_off[3] = {0, 0, 0}, nflat = 0;
    size_t packed_w_n = 0, packed_b_n = 0;
    int obs_feat = 0, plane = 0, H = 0, A = 0, S = 0;
    ActLayout lay{};
    int chain_buf[3][3][2];                 // LDS ping-pong buffers per chain

    float* d_flat = nullptr; float* d_Wp = nullptr; float* d_Bp = nullptr;
    int* d_srcW = nullptr; int* d_srcB = nullptr;
    int* d_plan[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};   // repr, pred, dyn, root, sim
    int* d_plan_sim_res = nullptr;          // register-resident image of the sim plan (or null)
    double* d_pbc = nullptr; double* d_sqrt = nullptr; float* d_aval = nullptr;
    double* d_pbterm = nullptr;             // pbc(Np) * (sqrt(Np) / (Nc + 1)), triangle
    size_t rtree_lds = 0;                                    // LDS of the LDS-cached ResNet tree step (0 = HBM kernel)
    float* d_bw = nullptr;                                   // host batch PER weights (mz_learner_step)
    float* d_rs_w = nullptr; float* d_per_cum = nullptr; float* d_per_p = nullptr;   // PER sampling
    long long* d_per_total = nullptr;
    int rs_last_B = 0;                                       // batch size of the last get_batch
    void* dp_comm = nullptr; int dp_world = 0, dp_rank = 0;  // mz_dp_init: RCCL communicator
    float* d_dp_cnt = nullptr;              // mz_train_run at world > 1: the finished-game count exchange
    char* d_tree = nullptr; size_t tree_game_bytes = 0; bool lds_tree = false; int dump_tree = 0;
    int time_nets = 0;                      // mz_debug_enable flag 2: events around each ResNet nets launch
    int time_unroll = 0;                    // flag 4: events around each ResNet learner unroll launch
                                            // (and each mz_learn_multi* launch)
    std::vector<hipEvent_t> tev; size_t tev_used = 0;
    bool use_res = false;                   // register-resident sim-plan kernel
    // small-batch kernel (mz_small.hip): schedule images + LDS layout
    bool small_ok = false;
    int n_cu = 256;
    int sm_n_sim = 0, sm_n_root = 0;
    float* d_sm_w = nullptr;                // [n_sim + n_root][2][256][16] weight image (sim then root)
    float* d_sm_bias = nullptr;             // [n_sim + n_root][2][64]
    // FC engines: a second image set (tile16 W/B, small W/bias) that the one-launch
    // learner step (mz_learn_small*) writes while its unroll reads the current set;
    // the host swaps the sets after the launch
    float* d_Wp2 = nullptr; float* d_Bp2 = nullptr; float* d_sm_w2 = nullptr; float* d_sm_bias2 = nullptr;
    int* d_sm_srcw = nullptr; int* d_sm_srcb = nullptr;
    size_t sm_w_n = 0, sm_b_n = 0;
    int* d_sm_rec[3] = {nullptr, nullptr, nullptr};   // per T in {1,2,4}
    int sm_lay[3][8];                       // per T: act_total, x_rep, x_pred, x_dyn, h_out, v_out, p_out, r_out
    size_t sm_lds[3] = {0, 0, 0};
    std::vector<uint32_t> sm_nzm;           // nonzero-chunk masks of the register images (SM_NZM_N)
    bool sm_bn = false;                     // BatchNorm FC layers: the bias image carries γ, β sections
    float* d_zero16 = nullptr;              // 64 zero bytes (sm_load's skipped chunks)
    unsigned* d_fault = nullptr;            // device fault word (MZ_FAULT_*), checked at host synchronisation
    int dbg_skip = -1;                      // debug: the hand-off producer that skips its publish
    unsigned long long poll_ticks = MZ_POLL_TICKS;
    int force_kernel = 0;                   // 0 auto, 1 tile16, 2 small
    // inverse image maps, one code per flat parameter: >= 0 position in the
    // weight image, <= -2 position -code-2 in the bias image, -1 none.  ADAM
    // scatters every update into the images through them (no repack).
    std::vector<int> inv_tile, inv_small;
    int* d_inv_tile = nullptr; int* d_inv_small = nullptr;
    std::string last_variant = "none";
    std::string last_lvariant = "none";     // the learner unroll's kernels (mz_learner_variant)
    int force_T = 0;                        // MZ_SMALL_T=1|2|4 (tests)
    float* d_hid = nullptr;
    float* d_obs = nullptr; uint8_t* d_legal = nullptr; int32_t* d_tp = nullptr;
    float* d_cv = nullptr; float* d_rv = nullptr; int32_t* d_act = nullptr;
    // learner
    float* d_m = nullptr; float* d_v = nullptr; float* d_grad = nullptr;
    double bp1 = 0.9, bp2 = 0.999;
    int bcap = 0;
    float *d_bobs = nullptr, *d_bact = nullptr, *d_btv = nullptr, *d_btr = nullptr, *d_btp = nullptr,
          *d_bgs = nullptr, *d_pv = nullptr, *d_pp = nullptr, *d_pr = nullptr, *d_loss = nullptr;
    double* d_sq = nullptr;                 // [3][MZ_L2_BLOCKS] partial Σθ²
    size_t* d_netoff = nullptr;             // [3] flat offset, [3] count per net
    unsigned* d_counter = nullptr;          // last-block counter of mz_learner_grad_kernel
    float* d_lterm = nullptr;               // [2][B(K+1)] loss terms
    unsigned long long* d_stamps = nullptr;
    // device self-play + replay shard (mz_selfplay.hip); own allocation list (re-init frees it)
    int sp_env = -1, sp_G = 0, sp_T = 0, sp_osz = 0, sp_cap = 0;
    uint8_t* d_sp_board = nullptr; int32_t* d_sp_player = nullptr; uint8_t* d_sp_over = nullptr;
    uint32_t* d_sp_ekey = nullptr; int sp_frames = 0;
    SpHist sp_hist{}, sp_ring{};
    long long* d_sp_counters = nullptr;
    int32_t* d_sp_done = nullptr; int32_t* d_sp_rpos = nullptr;
    float* d_sp_temp = nullptr;             // [G] per-slot temperatures (temperature_threshold)
    float* d_sp_tgame = nullptr;            // [G] each game's own temperature (mz_train_run)
    bool sp_latch = false;                  // mz_selfplay_move latches temperatures per game
    std::string tr_ckpt_path;               // mz_train_set_networks_path: periodic checkpoints
    int sp_eval = 0, sp_opp = MZ_OPP_SELF, sp_mzp = 1;    // mz_selfplay_mode
    long long* d_eval = nullptr;                          // [4] evaluation tally
    float* d_sp_dpow = nullptr;
    float *d_rs_obs = nullptr, *d_rs_act = nullptr, *d_rs_tv = nullptr, *d_rs_tr = nullptr, *d_rs_tp = nullptr,
          *d_rs_gs = nullptr;
    int32_t* d_rs_index = nullptr;
    int rs_cap = 0;
    bool sp_has_games = false;              // the FIFO never empties once a game is in
    bool sp_reset_pending = false;          // Atari-like env: the initial games start at the first move
    // get_batch one step ahead (the one-launch FC learner, PER off): the launch
    // for step t also samples step t+1's batch into the other batch set and
    // stamps that set's header {epoch, games played, step, B}; the next launch
    // uses a set only if its header still matches (the same shard state — a
    // stored game bumps `played` — step and B), else it samples in place.
    // Anything else that fills set 0 or re-creates the shard bumps the epoch.
    float *d_rs2_obs = nullptr, *d_rs2_act = nullptr, *d_rs2_tv = nullptr, *d_rs2_tr = nullptr,
          *d_rs2_tp = nullptr, *d_rs2_gs = nullptr;
    int32_t* d_rs2_index = nullptr;
    int pf_cap = 0, pf_cur = 0;
    long long* d_pf_hdr = nullptr;          // [2][4]
    long long pf_epoch = 1;
    // L learner steps per launch pair (mz_learner_train_multi_dev, ChainParams): the bank of
    // MZ_MULTI_MAX small-kernel images (θ_t .. θ_{t+L-1}), per-step batches, read-outs,
    // loss terms, Σθ² partials, fold counters and losses, for batches up to ml_cap
    float* d_bank_w = nullptr; float* d_bank_b = nullptr;
    // ResNet nets: the MFMA image bank (W, B), the flat-parameter bank, per-step unroll scratch (h, trunk
    // outputs), progress words and downsampled batches
    float* d_tbank_w = nullptr; float* d_tbank_b = nullptr; float* d_fbank = nullptr;
    float* d_ml_hs = nullptr; float* d_ml_ts = nullptr; float* d_ml_dsb = nullptr;
    unsigned long long* d_ml_prog = nullptr;
    unsigned long long ml_prog_epoch = 0;   // multi-step fused launches (d_ml_prog's prog_base = epoch · 64)
    int ml_cap = 0, ml_cap_L = 0, ml_last_B = 0, ml_last_L = 0, ml_last_R = 0;   // (ring: ensure_multi)
    float *d_ml_obs = nullptr, *d_ml_act = nullptr, *d_ml_tv = nullptr, *d_ml_tr = nullptr, *d_ml_tp = nullptr,
          *d_ml_gs = nullptr, *d_ml_pv = nullptr, *d_ml_pp = nullptr, *d_ml_pr = nullptr, *d_ml_terms = nullptr,
          *d_ml_out = nullptr;
    int32_t* d_ml_index = nullptr;
    double* d_ml_part = nullptr;
    unsigned* d_ml_cnt = nullptr;
    // actor–learner loop (mz_train_*): the actors' weight set (flat + the
    // search images), the queued nets (remote_NNs, flat), the learner step t
    struct WSet { float* flat = nullptr; float* Wp = nullptr; float* Bp = nullptr; float* smw = nullptr;
                  float* smb = nullptr; };
    WSet tr_actor;
    float* d_tr_queued = nullptr;
    int tr_B = 0;
    int64_t tr_t = 0, tr_games = 0, tr_refresh = 0;
    long long* h_tr_cnt = nullptr;          // pinned: num_played_games read back once per move
    long long* h_tr_pub = nullptr;          // coherent pinned: mz_tr_publish's {count, fault, sequence}
    long long tr_pub_seq = 0;
    // corrected-gradient learner (mz_backprop.hip): the unrolled graph and its arenas
    int learn_mode = MZ_LEARN_REF_SEMANTICS;
    bool bp_built = false;
    // the corrected learner for the ResNet nets (mz_rbp_sample / mz_rbp_dw)
    bool rbp_built = false;
    int rbp_n_app = 0, rbp_n_head = 0, rbp_arena = 0, rbp_obs_t = 0, rbp_dt = 0, rbp_xs = 0, rbp_n_job = 0, rbp_cap = 0;
    int rbp_ring = 0;                      // forward / backward LDS ring slots of mz_rbp_sample
    int2* d_rbp_gzero = nullptr; int rbp_n_gzero = 0;
    int rbp_threads = 256;
    int rbp_job0[4] = {0, 0, 0, 0};
    RbpApp* d_rbp_apps = nullptr; BpHead* d_rbp_heads = nullptr;
    RbpLayer* d_rbp_layers = nullptr; RbpUse* d_rbp_uses = nullptr; RbpJob* d_rbp_jobs = nullptr;
    float* d_rbp_act = nullptr; float* d_rbp_grad = nullptr;
    float* d_rbp_terms = nullptr; double* d_rbp_sq = nullptr;
    // ... through the downsampler (mz_dsbp_*): per-sample arenas, one dW job per conv output channel
    int dsbp_arena = 0, dsbp_dt = 0, dsbp_n_job = 0, dsbp_cap = 0;
    DsBpLayer* d_dsbp_lay = nullptr; DsDwJob* d_dsbp_jobs = nullptr;
    float* d_dsbp_act = nullptr; float* d_dsbp_grad = nullptr;
    int bp_n_app = 0, bp_n_head = 0, bp_n_job = 0, bp_tile_floats = 0, bp_obs_t = 0, bp_tiles_cap = 0;
    BpApp* d_bp_apps = nullptr; BpHead* d_bp_heads = nullptr; BpLayer* d_bp_layers = nullptr;
    BpUse* d_bp_uses = nullptr; BpJob* d_bp_jobs = nullptr;
    int2* d_bp_funits = nullptr; int* d_bp_flev = nullptr; int2* d_bp_bunits = nullptr; int* d_bp_blev = nullptr;
    int bp_n_flev = 0, bp_n_blev = 0, bp_n_funit = 0, bp_n_bunit = 0;
    int* d_bp_fsync = nullptr; int* d_bp_bsync = nullptr; int bp_cache_floats = 0, bp_obs_s = -1;
    double* d_bp_sq = nullptr; int bp_job0[4] = {0, 0, 0, 0};
    float* d_bp_act = nullptr; float* d_bp_grad = nullptr; float* d_bp_terms = nullptr;
    std::vector<void*> sp_allocs;
    std::vector<void*> allocs;
};

#define MZ_TRY(h, expr)                                                                  \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                \
            return -1;                                                                   \
        }                                                                                \
    } while (0)

static int fail(mz_handle* h, const std::string& m) { h->err = m; return -2; }
static int timing_events(mz_handle* h, hipEvent_t* e0, hipEvent_t* e1);

// Host-synchronous entry points (weights, state, replay read-outs, debug
// copies) wait for ALL of this process's work on the device, not only the
// handle's stream: `_dev` calls may have queued work on a caller stream
// (torch's, created non-blocking like the handle's), which a blocking
// hipMemcpy would not wait for.  A caller that orders its own
// work narrows the wait to one named stream plus the handle's own with
// mz_set_sync_stream, so unrelated device work is not waited for.
static hipError_t sync_device(mz_handle* h) {
    if (!h->sync_narrow) return hipDeviceSynchronize();
    hipError_t e = hipStreamSynchronize(h->sync_stream);
    return e != hipSuccess ? e : hipStreamSynchronize(h->stream);
}

// After a synchronisation: a kernel that gave up on a cross-workgroup publish
// (mz_poll_ge) left bits in d_fault; report them once (the word is cleared)
// as this call's error.  The outputs of the launches since the last check
// are then not to be trusted.
static int check_fault(mz_handle* h) {
    if (!h->d_fault) return 0;
    unsigned v = 0;
    MZ_TRY(h, hipMemcpy(&v, h->d_fault, 4, hipMemcpyDeviceToHost));
    if (!v) return 0;
    MZ_TRY(h, hipMemset(h->d_fault, 0, 4));
    char wait[32];
    std::snprintf(wait, sizeof(wait), "%.3g s", (double)h->poll_ticks / 1e8);   // the 100 MHz constant clock
    std::string m = std::string("device fault: a workgroup waited ") + wait + " for a publish that never came (";
    if (v & MZ_FAULT_RS_TRUNK) m += "mz_rsearch_nets trunk hand-off ";
    if (v & MZ_FAULT_RD_PROGRESS) m += "mz_runroll_fused_r chain progress ";
    h->err = m + "); the results of the launches since the last synchronisation are invalid (search results, "
                 "games self-play stored from them, losses, read-outs; the ref_semantics weights and ADAM state "
                 "do not read them and stay valid)";
    return -1;
}

// every host-synchronous call: wait (sync_device), then report a device fault
#define MZ_SYNC(h)                                    \
    do {                                              \
        MZ_TRY(h, sync_device(h));                    \
        if (check_fault(h)) return -1;                \
    } while (0)

template <typename T>
static hipError_t dalloc(mz_handle* h, T** p, size_t n) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T) + 16);
    if (e == hipSuccess) h->allocs.push_back(*p);
    return e;
}
// free one dalloc'd buffer before the handle is destroyed (the caller has drained the work using it)
static hipError_t dfree(mz_handle* h, void* p) {
    auto it = std::find(h->allocs.begin(), h->allocs.end(), p);
    if (it == h->allocs.end()) return hipErrorInvalidValue;
    h->allocs.erase(it);
    return hipFree(p);
}

// ------------------------------------------------------------ specs & plans
static void add_layer(mz_handle* h, int net, int chain, int in, int out, int act, bool bn = false) {
    LayerSpec L;
    L.net = net; L.chain = chain; L.in = in; L.out = out; L.act = act;
    L.flux_w = h->flat_off[net] + h->nparams[net]; h->nparams[net] += (size_t)in * out;
    L.flux_b = h->flat_off[net] + h->nparams[net]; h->nparams[net] += (size_t)out;
    if (bn) { L.bn = 1; L.flux_be = h->flat_off[net] + h->nparams[net]; h->nparams[net] += (size_t)2 * out; }
    L.nq = (in + 15) / 16;
    L.n_ob = (out + 15) / 16;
    L.packed_w = (int)h->packed_w_n; h->packed_w_n += (size_t)L.n_ob * 4 * L.nq * 64;
    // packed bias image: b, then (BatchNorm) γ and β, each n_ob*16 entries
    L.packed_b = (int)h->packed_b_n; h->packed_b_n += (size_t)L.n_ob * 16 * (bn ? 3 : 1);
    h->chains[net][chain].push_back((int)h->layers.size());
    h->layers.push_back(L);
}

// init_representation / init_prediction / init_dynamics (Learning.jl:87-142)
static void build_specs(mz_handle* h) {
    const mz_config& c = h->conf;
    const mz_ffhp& p = h->hp;
    const int W = c.observation_shape[0], Hh = c.observation_shape[1], C = c.observation_shape[2];
    const int hs = p.width_hidden, hid = p.hidden_state_size, A = c.action_space_size;
    h->obs_feat = W * Hh * (C * (c.stacked_observations + 1) + c.stacked_observations);   // :88
    h->plane = W * Hh;
    h->H = hid; h->A = A; h->S = c.num_iters;
    const bool bn = p.use_batch_norm != 0;                 // make_dense (Learning.jl:70-78)
    // repr
    h->flat_off[MZ_NET_REPR] = 0;
    add_layer(h, MZ_NET_REPR, CH_TRUNK, h->obs_feat, hs, MZ_ACT_RELU, bn);
    for (int i = 0; i < p.depth_representation; ++i) add_layer(h, MZ_NET_REPR, CH_TRUNK, hs, hs, MZ_ACT_RELU, bn);
    add_layer(h, MZ_NET_REPR, CH_TRUNK, hs, hid, MZ_ACT_IDENTITY);
    // pred
    h->flat_off[MZ_NET_PRED] = h->nparams[MZ_NET_REPR];
    add_layer(h, MZ_NET_PRED, CH_TRUNK, hid, hs, MZ_ACT_RELU, bn);
    for (int i = 0; i < p.depth_prediction; ++i) add_layer(h, MZ_NET_PRED, CH_TRUNK, hs, hs, MZ_ACT_RELU, bn);
    for (int i = 0; i < p.depth_value; ++i) add_layer(h, MZ_NET_PRED, CH_HEAD1, hs, hs, MZ_ACT_RELU, bn);
    add_layer(h, MZ_NET_PRED, CH_HEAD1, hs, 1, MZ_ACT_TANH);
    for (int i = 0; i < p.depth_policy; ++i) add_layer(h, MZ_NET_PRED, CH_HEAD2, hs, hs, MZ_ACT_RELU, bn);
    add_layer(h, MZ_NET_PRED, CH_HEAD2, hs, A, MZ_ACT_IDENTITY);
    // dyn
    h->flat_off[MZ_NET_DYN] = h->flat_off[MZ_NET_PRED] + h->nparams[MZ_NET_PRED];
    add_layer(h, MZ_NET_DYN, CH_TRUNK, W * Hh * (C + 1), hs, MZ_ACT_RELU, bn);                 // :120
    for (int i = 0; i < p.depth_dynamics; ++i) add_layer(h, MZ_NET_DYN, CH_TRUNK, hs, hs, MZ_ACT_RELU, bn);
    for (int i = 0; i < p.depth_state_head; ++i) add_layer(h, MZ_NET_DYN, CH_HEAD1, hs, hs, MZ_ACT_RELU, bn);
    add_layer(h, MZ_NET_DYN, CH_HEAD1, hs, hid, MZ_ACT_IDENTITY);
    for (int i = 0; i < p.depth_reward; ++i) add_layer(h, MZ_NET_DYN, CH_HEAD2, hs, hs, MZ_ACT_RELU, bn);
    add_layer(h, MZ_NET_DYN, CH_HEAD2, hs, 1, p.reward_activation);
    h->nflat = h->flat_off[MZ_NET_DYN] + h->nparams[MZ_NET_DYN];

    // LDS activation layout (floats), every region [rows][16]
    int off = 0;
    auto region = [&](int rows) { int o = off; off += rows * 16; return o; };
    auto in_rows = [&](int net) { return 16 * h->layers[h->chains[net][CH_TRUNK][0]].nq; };
    h->lay.rows_rep = in_rows(MZ_NET_REPR);
    h->lay.rows_pred = in_rows(MZ_NET_PRED);
    h->lay.rows_dyn = in_rows(MZ_NET_DYN);
    h->lay.x_pred = region(h->lay.rows_pred);
    h->lay.x_dyn = region(h->lay.rows_dyn);
    h->lay.h_out = region(mz_round16(hid));
    h->lay.v_out = region(16);
    h->lay.p_out = region(mz_round16(A));
    h->lay.r_out = region(16);
    auto chain_bufs = [&](int net) {
        for (int ch = 0; ch < 3; ++ch) {
            int rows = 0;
            for (int li : h->chains[net][ch]) rows = std::max(rows, 16 * h->layers[li].n_ob);
            if (rows == 0) { h->chain_buf[net][ch][0] = h->chain_buf[net][ch][1] = -1; continue; }
            h->chain_buf[net][ch][0] = region(rows);
            h->chain_buf[net][ch][1] = region(rows);
        }
    };
    chain_bufs(MZ_NET_PRED);
    // the representation (input + chain) only runs before / apart from the
    // dynamics net in every plan: they share one LDS union
    const int u0 = off;
    chain_bufs(MZ_NET_DYN);
    const int dyn_end = off;
    off = u0;
    h->lay.x_rep = region(h->lay.rows_rep);
    chain_bufs(MZ_NET_REPR);
    off = std::max(off, dyn_end);
    h->lay.total = off;
}

// Place chain `ch` of `net` in plan `pb` from stage `st0`; returns the end stage.
static int place_chain(mz_handle* h, PlanBuild& pb, int net, int ch, int st0, int in_first, int out_last) {
    const std::vector<int>& ls = h->chains[net][ch];
    const int n = (int)ls.size();
    pb.ensure(st0 + n);
    for (int i = 0; i < n; ++i) {
        const LayerSpec& S = h->layers[ls[i]];
        LayerDesc d;
        d.w_off = S.packed_w; d.b_off = S.packed_b; d.nq = S.nq; d.n_ob = S.n_ob; d.act = S.act; d.bn = S.bn;
        d.in_off = i == 0 ? in_first : h->chain_buf[net][ch][(i - 1) & 1];
        d.out_off = i == n - 1 ? out_last : h->chain_buf[net][ch][i & 1];
        d.out_rows = S.out;
        // value / reward heads' output activation is applied at read-out
        if (i == n - 1 && ch == CH_HEAD1 && net == MZ_NET_PRED) { h->lay.v_act = d.act; d.act = MZ_ACT_IDENTITY; }
        if (i == n - 1 && ch == CH_HEAD2 && net == MZ_NET_DYN) { h->lay.r_act = d.act; d.act = MZ_ACT_IDENTITY; }
        const int di = (int)pb.layers.size();
        pb.layers.push_back(d);
        for (int ob = 0; ob < S.n_ob; ++ob) pb.stages[st0 + i].push_back({di, ob});
    }
    return st0 + n;
}
static int trunk_out(mz_handle* h, int net) {
    const int n = (int)h->chains[net][CH_TRUNK].size();
    return h->chain_buf[net][CH_TRUNK][(n - 1) & 1];
}
// A two-headed net (pred / dyn) from stage st0 with trunk input `in`.
static int place_split_net(mz_handle* h, PlanBuild& pb, int net, int st0, int in) {
    const int t = place_chain(h, pb, net, CH_TRUNK, st0, in, trunk_out(h, net));
    const int to = trunk_out(h, net);
    int e1, e2;
    if (net == MZ_NET_PRED) {
        e1 = place_chain(h, pb, net, CH_HEAD1, t, to, h->lay.v_out);
        e2 = place_chain(h, pb, net, CH_HEAD2, t, to, h->lay.p_out);
    } else {
        e1 = place_chain(h, pb, net, CH_HEAD1, t, to, h->lay.h_out);
        e2 = place_chain(h, pb, net, CH_HEAD2, t, to, h->lay.r_out);
    }
    return std::max(e1, e2);
}

static int upload_plan(mz_handle* h, const PlanBuild& pb, int** dst) {
    std::vector<int> img = pb.image();
    MZ_TRY(h, dalloc(h, dst, img.size()));
    MZ_TRY(h, hipMemcpy(*dst, img.data(), img.size() * sizeof(int), hipMemcpyHostToDevice));
    return 0;
}

static int build_plans(mz_handle* h) {
    PlanBuild repr, pred, dyn, root, sim;
    place_chain(h, repr, MZ_NET_REPR, CH_TRUNK, 0, h->lay.x_rep, h->lay.h_out);
    place_split_net(h, pred, MZ_NET_PRED, 0, h->lay.x_pred);
    place_split_net(h, dyn, MZ_NET_DYN, 0, h->lay.x_dyn);
    const int e = place_chain(h, root, MZ_NET_REPR, CH_TRUNK, 0, h->lay.x_rep, h->lay.h_out);
    place_split_net(h, root, MZ_NET_PRED, e, h->lay.h_out);
    place_split_net(h, sim, MZ_NET_PRED, 0, h->lay.x_pred);
    place_split_net(h, sim, MZ_NET_DYN, 0, h->lay.x_dyn);
    const PlanBuild* all[5] = {&repr, &pred, &dyn, &root, &sim};
    for (int i = 0; i < 5; ++i)
        if (all[i]->stages.size() > MZ_MAX_STAGES) return fail(h, "network too deep for the plan executor");
    for (int i = 0; i < 5; ++i) if (upload_plan(h, *all[i], &h->d_plan[i])) return -1;
    // Register-resident image: the tasks of each stage go round-robin to the
    // 4 waves exactly as run_plan deals them; eligible when every wave has
    // <= MZ_RES_TASKS tasks of K <= 64 (nq <= 4).
    const int NW = MZ_THREADS / 64, NT = 16, RT = 9;    // MZ_RES_TASKS, ints per ResTask
    std::vector<std::vector<int>> per(NW);
    bool ok = true;
    for (int st = 0; st < (int)sim.stages.size(); ++st)
        for (int t = 0; t < (int)sim.stages[st].size(); ++t) {
            const LayerDesc& L = sim.layers[sim.stages[st][t].first];
            const int w = t % NW;
            if (L.nq > 4) ok = false;
            const int rt[RT] = {st, L.w_off, L.b_off, L.nq, sim.stages[st][t].second, L.act, L.in_off, L.out_off,
                                L.bn ? L.n_ob : 0};
            per[w].insert(per[w].end(), rt, rt + RT);
        }
    for (auto& v : per) if ((int)v.size() / RT > NT) ok = false;
    if (ok) {
        std::vector<int> img = {(int)sim.stages.size(), NT};
        for (auto& v : per) {
            img.push_back((int)v.size() / RT);
            img.insert(img.end(), v.begin(), v.end());
            img.resize(img.size() + (size_t)(NT * RT - (int)v.size()), 0);
        }
        MZ_TRY(h, dalloc(h, &h->d_plan_sim_res, img.size()));
        MZ_TRY(h, hipMemcpy(h->d_plan_sim_res, img.data(), img.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    return 0;
}


// ------------------------------------------------------------- small kernel
// Schedule the layers of one network set onto stages x 2 slots x 16 4-row
// blocks (mz_small.hip): list scheduling by longest remaining path; layers
// sharing a slot must have equal kq.  Returns false if not eligible.
struct SmSched {
    int n_stages = 0;
    std::vector<int> stage;            // per layer-in-set
    std::vector<int> slot, block0;
    std::vector<int> kq[SM_MAX_SIM > SM_MAX_ROOT ? SM_MAX_SIM : SM_MAX_ROOT];
};

static bool sm_schedule(const mz_handle* h, const std::vector<int>& set, const std::vector<std::vector<int>>& deps,
                        int max_stages, std::vector<int>& st, std::vector<int>& sl, std::vector<int>& b0,
                        std::vector<std::array<int, 2>>& stage_kq) {
    const int n = (int)set.size();
    std::vector<int> prio(n, 1);
    for (int it = 0; it < n; ++it)             // longest path to the end (deps point backwards)
        for (int i = 0; i < n; ++i)
            for (int d : deps[i]) prio[d] = std::max(prio[d], prio[i] + 1);
    st.assign(n, -1); sl.assign(n, -1); b0.assign(n, -1);
    stage_kq.clear();
    int done = 0;
    for (int s = 0; done < n; ++s) {
        if (s >= max_stages) return false;
        std::vector<int> ready;
        for (int i = 0; i < n; ++i) {
            if (st[i] >= 0) continue;
            bool ok = true;
            for (int d : deps[i]) ok &= st[d] >= 0 && st[d] < s;
            if (ok) ready.push_back(i);
        }
        std::stable_sort(ready.begin(), ready.end(), [&](int a, int b) { return prio[a] > prio[b]; });
        // 4 groups of 16 rows per slot: the 16 lanes of a DPP row serve the
        // 16 rows of one group and broadcast one shared input vector
        int fr[SM_SLOTS];
        for (int x = 0; x < SM_SLOTS; ++x) fr[x] = 4;
        std::array<int, 2> kq = {0, 0};
        for (int i : ready) {
            const LayerSpec& L = h->layers[set[i]];
            const int nb = (L.out + 15) / 16;
            for (int x = 0; x < SM_SLOTS; ++x)
                if (fr[x] >= nb) {
                    st[i] = s; sl[i] = x; b0[i] = 4 * (4 - fr[x]); fr[x] -= nb; ++done;   // b0 in 4-row units
                    break;
                }
        }
        stage_kq.push_back(kq);
    }
    return true;
}

static int build_small(mz_handle* h) {
    for (const LayerSpec& L : h->layers)
        if (L.in > 64 || L.out > 64) return 0;          // not eligible: tile-16 kernel only
    if (h->A > 16) return 0;
    // network sets: SIM = prediction + dynamics, ROOT = representation
    std::vector<int> sim, root;
    auto add_net = [&](std::vector<int>& set, int net) {
        for (int ch = 0; ch < 3; ++ch) for (int li : h->chains[net][ch]) set.push_back(li);
    };
    add_net(sim, MZ_NET_PRED); add_net(sim, MZ_NET_DYN); add_net(root, MZ_NET_REPR);
    auto deps_of = [&](const std::vector<int>& set) {
        std::vector<std::vector<int>> d(set.size());
        auto pos = [&](int li) { for (size_t i = 0; i < set.size(); ++i) if (set[i] == li) return (int)i; return -1; };
        for (size_t i = 0; i < set.size(); ++i) {
            const LayerSpec& L = h->layers[set[i]];
            const auto& chain = h->chains[L.net][L.chain];
            const int k = (int)(std::find(chain.begin(), chain.end(), set[i]) - chain.begin());
            if (k > 0) d[i].push_back(pos(chain[k - 1]));
            else if (L.chain != CH_TRUNK) d[i].push_back(pos(h->chains[L.net][CH_TRUNK].back()));
        }
        return d;
    };
    std::vector<int> st_s, sl_s, b0_s, st_r, sl_r, b0_r;
    std::vector<std::array<int, 2>> kq_s, kq_r;
    if (!sm_schedule(h, sim, deps_of(sim), SM_MAX_SIM, st_s, sl_s, b0_s, kq_s)) return 0;
    if (!sm_schedule(h, root, deps_of(root), SM_MAX_ROOT, st_r, sl_r, b0_r, kq_r)) return 0;
    h->sm_n_sim = (int)kq_s.size();
    h->sm_n_root = (int)kq_r.size();
    const int nrec = h->sm_n_sim + h->sm_n_root;
    // weight / bias gather images: [rec] stage images (sm_widx) and [rec][slot][row]; with
    // BatchNorm FC layers the bias image has two more sections of the same shape: γ, β
    bool any_bn = false;
    for (const LayerSpec& L : h->layers) any_bn |= L.bn != 0;
    h->sm_bn = any_bn;
    const size_t nri = (size_t)nrec * SM_SLOTS * 64;
    std::vector<int> sw((size_t)nrec * SM_SLOTS * 256 * 16, -1), sb(nri * (any_bn ? 3 : 1), -1);
    auto fill = [&](const std::vector<int>& set, const std::vector<int>& st, const std::vector<int>& sl,
                    const std::vector<int>& b0, int rec0) {
        for (size_t i = 0; i < set.size(); ++i) {
            const LayerSpec& L = h->layers[set[i]];
            const int kq = 4 * ((L.in + 15) / 16), r = rec0 + st[i];
            for (int row = 0; row < L.out; ++row) {
                const int srow = 4 * b0[i] + row;                       // slot row
                sb[((size_t)r * SM_SLOTS + sl[i]) * 64 + srow] = (int)(L.flux_b + row);
                if (L.bn) {
                    sb[nri + ((size_t)r * SM_SLOTS + sl[i]) * 64 + srow] = (int)(L.flux_be + L.out + row);   // γ
                    sb[2 * nri + ((size_t)r * SM_SLOTS + sl[i]) * 64 + srow] = (int)(L.flux_be + row);      // β
                }
                for (int q = 0; q < 4; ++q)
                    for (int j = 0; j < kq; ++j) {
                        const int k = q * kq + j;
                        if (k >= L.in) continue;
                        sw[sm_widx(r, sl[i], q, srow, j)] =
                            (int)(L.flux_w + row + (size_t)L.out * k);
                    }
            }
        }
    };
    fill(sim, st_s, sl_s, b0_s, 0);
    fill(root, st_r, sl_r, b0_r, h->sm_n_sim);
    h->sm_w_n = sw.size(); h->sm_b_n = sb.size();
    // nonzero-chunk masks (mz_small_params.h SM_NZM_N): per stage and wave,
    // bit q*4 + c set when any row of the wave's group gathers a weight into
    // chunk c of DPP row q
    h->sm_nzm.assign(SM_NZM_ALLOC, 0);        // zero padding past SM_NZM_N
    for (int r = 0; r < nrec; ++r)
        for (int sl2 = 0; sl2 < SM_SLOTS; ++sl2)
            for (int srow = 0; srow < 64; ++srow)
                for (int q = 0; q < 4; ++q)
                    for (int j = 0; j < 16; ++j)
                        if (sw[sm_widx(r, sl2, q, srow, j)] >= 0)
                            h->sm_nzm[(size_t)(sl2 * 4 + (srow >> 4)) * SM_NZM_ST + r] |= 1u << (q * 4 + j / 4);
    h->inv_small.assign(h->nflat, -1);
    for (size_t i = 0; i < sw.size(); ++i) if (sw[i] >= 0) h->inv_small[(size_t)sw[i]] = (int)i;
    for (size_t i = 0; i < sb.size(); ++i) if (sb[i] >= 0) h->inv_small[(size_t)sb[i]] = -(int)i - 2;
    MZ_TRY(h, dalloc(h, &h->d_zero16, 16));
    MZ_TRY(h, hipMemset(h->d_zero16, 0, 64));
    MZ_TRY(h, dalloc(h, &h->d_sm_srcw, sw.size()));
    MZ_TRY(h, dalloc(h, &h->d_sm_srcb, sb.size()));
    MZ_TRY(h, dalloc(h, &h->d_sm_w, sw.size()));
    MZ_TRY(h, dalloc(h, &h->d_sm_bias, sb.size()));
    MZ_TRY(h, hipMemcpy(h->d_sm_srcw, sw.data(), sw.size() * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_sm_srcb, sb.data(), sb.size() * 4, hipMemcpyHostToDevice));
    // per-T LDS layouts and records
    const int Ts[3] = {1, 2, 4};
    for (int ti = 0; ti < 3; ++ti) {
        const int T = Ts[ti];
        int off = 0;
        auto region = [&](int rows) { int o = off; off += (rows * T + 3) / 4 * 4; return o; };
        // every input buffer has 64 rows (zero beyond K): the kernel runs 16
        // steps per quarter and reads rows up to 3*kq + 15 < 64
        int* lay = h->sm_lay[ti];
        lay[1] = region(64);
        lay[2] = region(64);
        lay[3] = region(64);
        lay[4] = region(h->H);
        lay[5] = region(1);
        lay[6] = region(h->A);
        lay[7] = region(1);
        int cb[3][3][2];
        for (int net = 0; net < 3; ++net)
            for (int ch = 0; ch < 3; ++ch) { cb[net][ch][0] = region(64); cb[net][ch][1] = region(64); }
        lay[0] = off;
        auto io = [&](int li, int& in_off, int& out_off) {
            const LayerSpec& L = h->layers[li];
            const auto& chain = h->chains[L.net][L.chain];
            const int k = (int)(std::find(chain.begin(), chain.end(), li) - chain.begin());
            const int n = (int)chain.size();
            const auto& trunk = h->chains[L.net][CH_TRUNK];
            const int trunk_out = cb[L.net][CH_TRUNK][((int)trunk.size() - 1) & 1];
            if (k > 0) in_off = cb[L.net][L.chain][(k - 1) & 1];
            else if (L.chain != CH_TRUNK) in_off = trunk_out;
            else in_off = L.net == MZ_NET_REPR ? lay[1] : L.net == MZ_NET_PRED ? lay[2] : lay[3];
            if (k < n - 1) out_off = cb[L.net][L.chain][k & 1];
            else if (L.chain == CH_TRUNK) out_off = L.net == MZ_NET_REPR ? lay[4] : trunk_out;
            else if (L.net == MZ_NET_PRED) out_off = L.chain == CH_HEAD1 ? lay[5] : lay[6];
            else out_off = L.chain == CH_HEAD1 ? lay[4] : lay[7];
        };
        // int4 per [stage][slot][row]: {input base, kq, out | relu << 30 (-1 =
        // unused), bias (filled on device)}; unused rows read offset 0 with
        // zero weights
        std::vector<int> rec((size_t)nrec * SM_REC_INTS, 0);
        for (size_t i = 0; i < rec.size(); i += 4) rec[i + 2] = -1;
        auto rec_fill = [&](const std::vector<int>& set, const std::vector<int>& st, const std::vector<int>& sl,
                            const std::vector<int>& b0, int rec0) {
            for (size_t i = 0; i < set.size(); ++i) {
                const LayerSpec& L = h->layers[set[i]];
                int in_off, out_off;
                io(set[i], in_off, out_off);
                int* R = rec.data() + (size_t)(rec0 + st[i]) * SM_REC_INTS;
                const int kq = 4 * ((L.in + 15) / 16);
                // every row of the layer's 16-row groups carries the input base
                // and kq (the DPP row broadcasts them); rows beyond L.out have
                // zero weights and no output
                const int rows = (L.out + 15) / 16 * 16;
                for (int row = 0; row < rows; ++row) {
                    int* e = R + 4 * (sl[i] * 64 + 4 * b0[i] + row);
                    e[0] = in_off;
                    e[1] = kq;
                    e[2] = row < L.out ? (out_off + row * T) | (L.act == MZ_ACT_RELU ? 1 << 30 : 0) |
                                             (L.bn ? 1 << 29 : 0) : -1;
                }
            }
        };
        rec_fill(sim, st_s, sl_s, b0_s, 0);
        rec_fill(root, st_r, sl_r, b0_r, h->sm_n_sim);
        MZ_TRY(h, dalloc(h, &h->d_sm_rec[ti], rec.size()));
        MZ_TRY(h, hipMemcpy(h->d_sm_rec[ti], rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
        const int S = h->S, NN = S + 1, PS = 2 * (S + 2);
        size_t ints = (size_t)lay[0] + (size_t)(nrec + 1) * SM_REC_INTS +
                      ((size_t)T * NN * h->H + 3) / 4 * 4 + 296 + ((size_t)T * PS + 3) / 4 * 4 +
                      (size_t)4 * (S + 2) + MZ_MAX_ACTIONS;
        // + the pb_term triangle (the small kernel requires it in LDS; when
        // the total exceeds the LDS budget the tile-16 kernel is used)
        h->sm_lds[ti] = ints * 4 + (size_t)T * h->tree_game_bytes + pbterm_count(S) * 8 +
                        // the cached select: entries, path levels, N per slot, tags
                        (size_t)T * (8 * NN + 8 * (S + 2) + 4 * NN) + 16 + 4 * 16 + 4 * 8 + 4 * 4 +
                        (any_bn ? nri * 8 : 0);                          // BatchNorm (γ, β) per record row
    }
    return 1;
}

// MFMA fragment image: packed W [ob][ks][lane] <- W[ob*16 + (lane&15)][ks*4 + (lane>>4)]
// (Flux W is (out,in) column-major: element (o,i) at flux_w + o + out*i).
static int build_pack_index(mz_handle* h) {
    std::vector<int> sw(h->packed_w_n, -1), sb(h->packed_b_n, -1);
    for (const LayerSpec& L : h->layers) {
        const int nks = 4 * L.nq;
        for (int ob = 0; ob < L.n_ob; ++ob)
            for (int ks = 0; ks < nks; ++ks)
                for (int lane = 0; lane < 64; ++lane) {
                    const int o = ob * 16 + (lane & 15), k = ks * 4 + (lane >> 4);
                    const size_t dst = (size_t)L.packed_w + ((size_t)ob * nks + ks) * 64 + lane;
                    if (o < L.out && k < L.in) sw[dst] = (int)(L.flux_w + o + (size_t)L.out * k);
                }
        for (int o = 0; o < L.out; ++o) sb[(size_t)L.packed_b + o] = (int)(L.flux_b + o);
        if (L.bn)                                   // γ, β after the bias (LayerDesc.bn)
            for (int o = 0; o < L.out; ++o) {
                sb[(size_t)L.packed_b + L.n_ob * 16 + o] = (int)(L.flux_be + L.out + o);
                sb[(size_t)L.packed_b + 2 * L.n_ob * 16 + o] = (int)(L.flux_be + o);
            }
    }
    h->inv_tile.assign(h->nflat, -1);
    for (size_t i = 0; i < sw.size(); ++i) if (sw[i] >= 0) h->inv_tile[(size_t)sw[i]] = (int)i;
    for (size_t i = 0; i < sb.size(); ++i) if (sb[i] >= 0) h->inv_tile[(size_t)sb[i]] = -(int)i - 2;
    MZ_TRY(h, dalloc(h, &h->d_srcW, sw.size()));
    MZ_TRY(h, dalloc(h, &h->d_srcB, sb.size()));
    MZ_TRY(h, hipMemcpy(h->d_srcW, sw.data(), sw.size() * sizeof(int), hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_srcB, sb.data(), sb.size() * sizeof(int), hipMemcpyHostToDevice));
    return 0;
}

static int repack(mz_handle* h, hipStream_t st = nullptr) {
    const int T = 256;
    if (!st) st = h->stream;
    hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_w_n + T - 1) / T)), dim3(T), 0, st,
                       h->d_flat, h->d_srcW, h->d_Wp, h->packed_w_n);
    if (h->packed_b_n)
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_b_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_srcB, h->d_Bp, h->packed_b_n);
    if (h->small_ok) {
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_w_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_sm_srcw, h->d_sm_w, h->sm_w_n);
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_b_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_sm_srcb, h->d_sm_bias, h->sm_b_n);
    }
    if (h->d_sm_w2) {                            // the second image set (one-launch learner step)
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_w_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_srcW, h->d_Wp2, h->packed_w_n);
        if (h->packed_b_n)
            hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_b_n + T - 1) / T)), dim3(T), 0, st,
                               h->d_flat, h->d_srcB, h->d_Bp2, h->packed_b_n);
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_w_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_sm_srcw, h->d_sm_w2, h->sm_w_n);
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_b_n + T - 1) / T)), dim3(T), 0, st,
                           h->d_flat, h->d_sm_srcb, h->d_sm_bias2, h->sm_b_n);
    }
    MZ_TRY(h, hipGetLastError());
    return 0;
}

// LDS of mz_unroll_small{1,2}: activations, records (+1 slack stage), staging
static size_t unroll_small_lds(const mz_handle* h, int ti) {
    const size_t nri = (size_t)(h->sm_n_sim + h->sm_n_root) * SM_SLOTS * 64;
    return ((size_t)h->sm_lay[ti][0] + (size_t)(h->sm_n_sim + h->sm_n_root + 1) * SM_REC_INTS + 64) * 4 +
           (h->sm_bn ? nri * 8 : 0);                                   // BatchNorm (γ, β) per record row
}

static size_t tree_game_bytes(int S, int A) {
    return tree_bytes((S + 1) * A, S + 1);
}
static size_t search_lds_base(const mz_handle* h) {
    return (size_t)h->lay.total * 4 + (size_t)(416 + 16 * 2 * (h->S + 2)) * 4;
}
static size_t search_lds_bytes(const mz_handle* h) {
    return search_lds_base(h) + (h->lds_tree ? (size_t)MZ_TILE * h->tree_game_bytes : 0);
}

typedef void (*search_fn)(SearchParams);
static search_fn search_kernel(const mz_handle* h) {
    if (h->use_res) return h->lds_tree ? mz_search_kernel_lds_res : mz_search_kernel_hbm_res;
    return h->lds_tree ? mz_search_kernel_lds : mz_search_kernel_hbm;
}

// ------------------------------------------------------------------- ABI
extern "C" {

const char* mz_create_error(void) { return g_create_error.c_str(); }
const char* mz_last_error(const mz_handle* h) { return h ? h->err.c_str() : g_create_error.c_str(); }

// ------------------------------------------------------------- ResNet nets
// Row a14: the intended architecture of Learning.jl:148-255,
// op for op as oracle/mz_oracle.c onet_build_resnet, in Flux.params order:
// Conv weight (kw,kh,cin,cout) col-major, bias, BatchNorm β, γ; Dense W
// (out,in) col-major, b.
struct RSpec {
    int chain, conv, cin, cout, kw, kh, act, bn, res_save, res_add;
    size_t woff, boff, bnoff;               // local to the net
};

static std::vector<RSpec> rn_specs(const mz_config& c, const mz_resnet_hp& hp, int net, size_t* nparams) {
    const int W = c.observation_shape[0], H = c.observation_shape[1], C = c.observation_shape[2];
    const int nf = hp.num_filters, nb = hp.num_blocks, hs = hp.width_hidden, A = c.action_space_size;
    const int P = W * H, nvf = hp.num_first_head_filters, npf = hp.num_second_head_filters;
    std::vector<RSpec> v;
    size_t n = 0;
    auto conv = [&](int ch, int cin, int cout, int kw, int kh) {
        RSpec r{ch, 1, cin, cout, kw, kh, MZ_ACT_RELU, 1, 0, 0, 0, 0, 0};
        r.woff = n; n += (size_t)kw * kh * cin * cout;
        r.boff = n; n += (size_t)cout;
        r.bnoff = n; n += (size_t)2 * cout;
        v.push_back(r);
    };
    auto block = [&](int ch, int f, int k) { conv(ch, f, f, k, k); v.back().res_save = 1; conv(ch, f, f, k, k);
                                             v.back().res_add = 1; };
    auto dense = [&](int ch, int in, int out, int act) {
        RSpec r{ch, 0, in, out, 1, 1, act, 0, 0, 0, 0, 0, 0};
        r.woff = n; n += (size_t)in * out;
        r.boff = n; n += (size_t)out;
        v.push_back(r);
    };
    if (net == MZ_NET_REPR) {
        const int kw = hp.conv_kernel_size[0], kh = hp.conv_kernel_size[1];
        conv(0, C * (c.stacked_observations + 1) + c.stacked_observations, nf, kw, kh);
        for (int i = 0; i < nb; ++i) block(0, nf, kw);
    } else if (net == MZ_NET_PRED) {
        conv(0, nf, nf, 1, 1);
        for (int i = 0; i < nb; ++i) block(0, nf, 1);
        conv(1, nf, nvf, 1, 1);
        dense(1, P * nvf, hs, MZ_ACT_RELU);
        for (int i = 0; i < hp.depth_value; ++i) dense(1, hs, hs, MZ_ACT_RELU);
        dense(1, hs, 1, MZ_ACT_TANH);
        conv(2, nf, npf, 1, 1);
        dense(2, P * npf, hs, MZ_ACT_IDENTITY);
        for (int i = 0; i < hp.depth_value; ++i) dense(2, hs, hs, MZ_ACT_RELU);    // :222 depth_value
        dense(2, hs, A, MZ_ACT_IDENTITY);
    } else {
        conv(0, nf + 1, nf, 1, 1);
        for (int i = 0; i < nb; ++i) block(0, nf, 1);
        conv(1, nf, nf, 1, 1);
        for (int i = 0; i < nb; ++i) block(1, nf, 1);
        conv(2, nf, nvf, 1, 1);
        dense(2, P * nvf, hs, MZ_ACT_RELU);
        for (int i = 0; i < hp.depth_value; ++i) dense(2, hs, hs, MZ_ACT_RELU);
        dense(2, hs, 1, hp.reward_activation);
    }
    *nparams = n;
    return v;
}

// LDS plan of one net for a tile of NG games (floats).  Trunk: X -> B0, each
// block B0 -> B1 -> B0 (residual in place); head 1 reads B0 (the dynamics
// state head runs its tower in B2 / B1, B2 aliasing the dead input X); head 2
// reads B0 through the small buffers S0..S2; outputs O0 / O1.
// Offset table of a narrow plan's layer L with a kernel > 1x1 (MODE 4 of
// rn_layer_t): for quarter q, chunk c, column n < ncols_t and bank slot
// sl = ((n >> 2) & 3) ^ σ(kl), the byte addresses of B(k, n), k = (q·nq + 4c +
// jj)·4 + kl, jj = 0..3 — the same operand MODE 2 gathers through the k table —
// or of the zero float for taps off the board, padded steps and columns past
// the tile.  One 16-byte read gives a lane a chunk's four addresses.
static void rn_otab_fill(std::vector<int>& t, const RLayer& L, int NG, int W, int P, int ncols_t, int zero_off) {
    static const int sinv[4] = {0, 2, 3, 1};                      // σ^-1, σ = (0, 3, 1, 2)
    const int nch = ((L.nq + 3) & ~3) / 4;
    for (int q = 0; q < 4; ++q)
        for (int c = 0; c < nch; ++c)
            for (int n = 0; n < ncols_t; ++n)
                for (int sl = 0; sl < 4; ++sl)
                    for (int jj = 0; jj < 4; ++jj) {
                        const int kl = sinv[sl ^ ((n >> 2) & 3)], j = 4 * c + jj, k = (q * L.nq + j) * 4 + kl;
                        int a = zero_off;
                        if (j < L.nq && k < L.K && n < P * NG) {
                            const int ci = k / L.kk, r = k - ci * L.kk, jy = r / L.kw, ix = r - jy * L.kw;
                            const int dx = (L.kw - 1 - ix) - L.pw, dy = (L.kh - 1 - jy) - L.ph;
                            const int p = n / NG, g = n - p * NG, px = p % W + dx, py = p / W + dy;
                            if (px >= 0 && px < W && py >= 0 && py < P / W)
                                a = L.in_off + ci * P * NG + (px + W * py) * NG + g;
                        }
                        t.push_back(a * 4);
                    }
}

// mz_runroll_chain_r[3] applies when the dynamics chain ([0, dyn_split)) is
// RD_NL (one column block) or RD_NL3 (three column blocks) 1x1 conv layers of
// 64 channels with BatchNorm + relu: layer 0 on the plain input with 4 < nq <=
// 8 (nf + 1 channels: two A chunks), the others K = 64 on k-blocked inputs
static size_t rd_chain_lds(const mz_handle* h) { return h->rn_lds_l + (size_t)h->rn_dyn_split * 64 * 16; }
static int rd_chain_ok(const mz_handle* h) {          // the column blocks, or 0
    const RPlan& R = h->rplan_l[MZ_NET_DYN];
    const int nb = (h->plane * h->rn_ng_l + 15) / 16;
    // (three blocks / 18 layers: 304 resident VGPRs, the kernel spills — measured 1.27k vs 1.53k learner
    // steps/s on Connect4 ResNet-8 — so only on request, MZ_RN_RD3=1)
    static const bool rd3 = std::getenv("MZ_RN_RD3") != nullptr;
    if (!((nb == 1 && h->rn_dyn_split == RD_NL) || (rd3 && nb == 3 && h->rn_dyn_split == RD_NL3))) return 0;
    for (int i = 0; i < h->rn_dyn_split; ++i) {
        const RLayer& L = R.L[i];
        if (L.kk != 1 || L.cout != 64 || L.n_ob != 4 || !L.spatial || !L.bn || L.act != MZ_ACT_RELU) return 0;
        if (i == 0 ? (L.in_kb || L.nq <= 4 || L.nq > 8) : (!L.in_kb || L.K != 64 || L.nq != 4)) return 0;
    }
    return rd_chain_lds(h) <= kLdsMax ? nb : 0;
}
// mz_runroll_pred_r applies when the prediction trunk ([0, RP_NL), the
// first head layer next) is RP_NL such layers, all on k-blocked inputs
static size_t rp_pred_lds(const mz_handle* h) { return h->rn_lds_l + (size_t)RP_NL * 64 * 16; }
static bool rp_pred_ok(const mz_handle* h) {
    const RPlan& R = h->rplan_l[MZ_NET_PRED];
    if ((h->plane * h->rn_ng_l + 15) / 16 != 1 || R.n <= RP_NL || R.L[RP_NL].cout == 64) return false;
    if (2 * h->rhp.num_blocks + 1 != RP_NL) return false;
    for (int i = 0; i < RP_NL; ++i) {
        const RLayer& L = R.L[i];
        if (L.kk != 1 || L.cout != 64 || L.n_ob != 4 || !L.spatial || !L.bn || L.act != MZ_ACT_RELU ||
            !L.in_kb || L.K != 64 || L.nq != 4)
            return false;
    }
    // the heads in rn_specs order: value [RP_NL, RP_NL + nv), policy after (the fused
    // launch runs them in separate blocks)
    const int nv = 3 + h->rhp.depth_value;
    if (R.n != RP_NL + 2 * nv || R.L[RP_NL].cout != h->rhp.num_first_head_filters ||
        R.L[RP_NL + nv].cout != h->rhp.num_second_head_filters || R.L[RP_NL + nv - 1].cout != 1)
        return false;
    return rp_pred_lds(h) <= kLdsMax;
}

static RPlan rn_plan(const mz_handle* h, const std::vector<RSpec>& sp, int net, int NG, size_t flat_off,
                     int& w_img, std::vector<int>* srcw, bool sep_b2 = false, std::vector<int>* otab = nullptr) {
    const mz_config& c = h->rconf;
    const int W = c.observation_shape[0], Hh = c.observation_shape[1], P = W * Hh;
    const int nf = h->rhp.num_filters, hs = h->rhp.width_hidden;
    const int in_feat = net == MZ_NET_REPR ? h->rin_feat : net == MZ_NET_PRED ? h->H : h->H + h->plane;
    const int big = nf * P * NG;
    int off = 0;
    auto region = [&](int n) { int o = off; off += (n + 3) / 4 * 4; return o; };
    RPlan R;
    std::memset(&R, 0, sizeof(R));
    // the dynamics state head's B2 aliases the dead input X, or (sep_b2, when the
    // LDS allows) has its own region, so that its layout can be k-blocked
    const int X = region(std::max(in_feat * NG, net == MZ_NET_DYN && !sep_b2 ? big : 0));
    const int B0 = region(big), B1 = region(big);
    // (aliased, B2 sits at the END of X's region, at a different offset from X:
    // a region's layout follows the readers of its offset, so B2 can be
    // k-blocked for the state head's 1x1 convs while X stays plain for the
    // K = nf + 1 first layer; X is dead once that layer has run)
    const int xsz = (std::max(in_feat * NG, net == MZ_NET_DYN && !sep_b2 ? big : 0) + 3) / 4 * 4;
    const int B2 = net == MZ_NET_DYN && sep_b2 ? region(big) : X + (xsz - big) / 4 * 4;
    int headc = 0;
    for (const RSpec& r : sp) if (r.chain && r.conv && r.cout != nf) headc = std::max(headc, r.cout * P * NG);
    const int S0 = region(std::max(headc, hs * NG)), S1 = region(hs * NG), S2 = region(hs * NG);
    const int O0 = net == MZ_NET_PRED ? region(NG) : B0;             // REPR / DYN out0 = h (B0 / B2)
    const int O1 = net == MZ_NET_REPR ? 0 : region((net == MZ_NET_PRED ? h->A : 1) * NG);
    R.in_off = X; R.in_feat = in_feat;
    int cur[3] = {X, B0, B0};                                        // current input of each chain
    int ping[3] = {0, S1, S1};
    for (size_t i = 0; i < sp.size(); ++i) {
        const RSpec& r = sp[i];
        RLayer& L = R.L[R.n++];
        L.kk = r.kw * r.kh; L.kw = r.kw; L.kh = r.kh; L.pw = r.kw / 2; L.ph = r.kh / 2;
        L.K = r.conv ? r.kw * r.kh * r.cin : r.cin;
        L.cout = r.cout; L.nq = (L.K + 15) / 16; L.n_ob = (r.cout + 15) / 16;
        L.spatial = r.conv; L.act = r.act; L.bn = r.bn; L.res_add = r.res_add;
        L.boff = (int)(flat_off + r.boff); L.bnoff = (int)(flat_off + r.bnoff);
        L.ktab = -1;
        L.in_off = cur[r.chain];
        const bool last_in_chain = i + 1 == sp.size() || sp[i + 1].chain != r.chain;
        if (r.chain == 0) {
            if (r.res_add) { L.out_off = B0; L.res_off = B0; L.in_off = B1; }
            else if (r.res_save) L.out_off = B1;
            else L.out_off = B0;
            cur[0] = r.res_save ? B1 : B0;
            if (r.res_add) cur[0] = B0;
            if (last_in_chain) { cur[1] = cur[2] = B0; }
        } else if (r.chain == 1 && net == MZ_NET_DYN) {            // state head tower in B2 / B1
            if (r.res_add) { L.in_off = B1; L.out_off = B2; L.res_off = B2; }
            else if (r.res_save) { L.out_off = B1; }
            else L.out_off = B2;
            cur[1] = r.res_save ? B1 : B2;
        } else {                                                    // conv head -> Dense chain
            if (last_in_chain) L.out_off = r.chain == 1 ? O0 : O1;
            else if (r.conv) L.out_off = S0;
            else { L.out_off = ping[r.chain]; ping[r.chain] = ping[r.chain] == S1 ? S2 : S1; }
            cur[r.chain] = L.out_off;
        }
        // A fragments [ob][q][j/4][lane][j%4] (NQ padded to NQ4 = 4⌈NQ/4⌉ with
        // zeros): one 16-byte load gives a lane four k-steps of a quarter chain
        L.w_img = w_img;
        const int nq4 = (L.nq + 3) & ~3;
        for (int ob = 0; ob < L.n_ob; ++ob)
            for (int q = 0; q < 4; ++q)
                for (int jc = 0; jc < nq4 / 4; ++jc)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int jj = 0; jj < 4; ++jj) {
                            const int j = 4 * jc + jj;
                            const int o = ob * 16 + (lane & 15), k = (q * L.nq + j) * 4 + (lane >> 4);
                            int src = -1;
                            if (j < L.nq && o < r.cout && k < L.K)
                                src = (int)(flat_off + r.woff + (r.conv ? (size_t)k + (size_t)L.K * o
                                                                        : (size_t)o + (size_t)r.cout * k));
                            if (srcw) srcw->push_back(src);
                        }
        w_img += L.n_ob * 4 * nq4 * 64;
        // epilogue image: per output row o, {bias, γ, β, 0} (a lane's four rows
        // are four 16-byte loads; ADAM scatters into it through the same inverse map)
        L.ep_img = w_img;
        for (int o = 0; o < L.n_ob * 16; ++o) {
            const bool in = o < r.cout;
            const int e[4] = {in ? (int)(flat_off + r.boff + o) : -1,
                              in && r.bn ? (int)(flat_off + r.bnoff + r.cout + o) : -1,
                              in && r.bn ? (int)(flat_off + r.bnoff + o) : -1, -1};
            if (srcw) for (int x = 0; x < 4; ++x) srcw->push_back(e[x]);
        }
        w_img += L.n_ob * 16 * 4;
        if (L.kk > 1 && !otab) L.ktab = region(L.K);
    }
    // layouts, per LDS region: k-blocked when every layer that reads the region
    // as its B operand is a 1x1 conv / Dense with K % 64 == 0 (a region's
    // layout never changes, so in-place residual blocks and aliased regions
    // stay consistent); the final outputs are checked plain below
    auto capable = [&](const RLayer& L) { return L.kk == 1 && L.K % 64 == 0; };
    auto kb = [&](int off) {
        bool any = false, all = true;
        for (int j = 0; j < R.n; ++j)
            if (R.L[j].in_off == off) { any = true; all &= capable(R.L[j]); }
        return (int)(any && all);
    };
    R.in_kb = kb(X);
    for (int j = 0; j < R.n; ++j) {
        R.L[j].in_kb = kb(R.L[j].in_off);
        R.L[j].out_kb = kb(R.L[j].out_off);
        R.L[j].res_kb = R.L[j].res_add ? kb(R.L[j].res_off) : 0;
    }
    if (net == MZ_NET_REPR) { R.out0_off = B0; R.out0_n = h->H; R.out1_n = 0; }
    else if (net == MZ_NET_PRED) { R.out0_off = O0; R.out0_n = 1; R.out1_off = O1; R.out1_n = h->A; }
    else { R.out0_off = B2; R.out0_n = h->H; R.out1_off = O1; R.out1_n = 1; }
    R.out0_act = R.out1_act = MZ_ACT_IDENTITY;
    for (int j = 0; j < R.n; ++j) {
        if (R.L[j].out_off == R.out0_off) R.out0_act = R.L[j].act;
        if (R.out1_n && R.L[j].out_off == R.out1_off) R.out1_act = R.L[j].act;
    }
    if (otab) {   // narrow plans: offset tables for the kernels > 1x1 (shared by layers of the same input / shape)
        const int n_nb = (P * NG + 15) >> 4, nbw = n_nb == 1 ? 1 : n_nb == 2 ? 2 : 3;
        const int ncols_t = (n_nb + nbw - 1) / nbw * nbw * 16;
        const int zero = region(4);
        std::vector<int> t;
        std::vector<std::pair<std::vector<int>, int>> seen;      // (in_off, K, kw, kh) -> table offset in t
        for (int i = 0; i < R.n; ++i) {
            RLayer& L = R.L[i];
            if (L.kk == 1) continue;
            const std::vector<int> key = {L.in_off, L.K, L.kw, L.kh};
            int at = -1;
            for (auto& e : seen) if (e.first == key) at = e.second;
            if (at < 0) { at = (int)t.size(); seen.push_back({key, at}); rn_otab_fill(t, L, NG, W, P, ncols_t, zero); }
            L.ktab = at;                                           // relative until the region is placed
            L.otab = 1;
        }
        if (!t.empty() && (size_t)(off + t.size() + 16 * 16 * 4) * 4 <= kLdsMax) {
            R.tab_lds = region((int)t.size());
            R.tab_n = (int)t.size();
            R.tab_src = (int)otab->size();
            R.zero_off = zero;
            otab->insert(otab->end(), t.begin(), t.end());
            for (int i = 0; i < R.n; ++i) if (R.L[i].otab) R.L[i].ktab += R.tab_lds;
        } else {                                                   // does not fit: the k-table gather (MODE 2)
            for (int i = 0; i < R.n; ++i) if (R.L[i].otab) { R.L[i].otab = 0; R.L[i].ktab = -1; }
        }
        for (int i = 0; i < R.n; ++i)                              // k tables for the layers that still need one
            if (R.L[i].kk > 1 && !R.L[i].otab && R.L[i].ktab < 0) R.L[i].ktab = region(R.L[i].K);
    }
    region(16 * 16 * 4);           // slack: past-the-tile lanes of k-blocked reads (MODE 3) read up to 15 columns on
    R.n_ktab = 0;
    for (int j = 0; j < R.n; ++j) R.n_ktab += R.L[j].kk > 1 && !R.L[j].otab;
    R.lds_floats = off;
    R.out0_kb = kb(R.out0_off);
    for (int j = 0; j < R.n; ++j) R.k[j] = rn_rk_pack(R.L[j]);
    if ((R.out0_kb && net == MZ_NET_PRED) || (R.out1_n && kb(R.out1_off))) R.n = -1;   // (never: read as plain)
    return R;
}

// pUCT tables (libm log2/sqrt on the host: the values the oracle computes
// inline), the action-plane values a/|A|, and the pb_term triangle
static int alloc_search_tables(mz_handle* h) {
    const mz_config& c = h->conf;
    const int S = h->S, A = h->A;
    std::vector<double> pbc(S + 2), sq(S + 2);
    for (int n = 0; n < S + 2; ++n) {
        pbc[n] = std::log2((double)(n + c.pb_c_base + 1) / (double)c.pb_c_base) + (double)c.pb_c_init;
        sq[n] = std::sqrt((double)n);
    }
    std::vector<float> av(A);
    for (int a = 0; a < A; ++a) av[a] = (float)((double)(a + 1) / (double)A);
    std::vector<double> pbt(pbterm_count(S), 0.0);
    for (int np = 0; np <= S + 1; ++np)
        for (int nc = 0; nc <= np; ++nc) pbt[pbterm_index(np, nc)] = pbc[np] * (sq[np] / (double)(nc + 1));
    MZ_TRY(h, dalloc(h, &h->d_pbc, pbc.size()));
    MZ_TRY(h, dalloc(h, &h->d_sqrt, sq.size()));
    MZ_TRY(h, dalloc(h, &h->d_aval, av.size()));
    MZ_TRY(h, dalloc(h, &h->d_pbterm, pbt.size()));
    MZ_TRY(h, hipMemcpy(h->d_pbc, pbc.data(), pbc.size() * 8, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_sqrt, sq.data(), sq.size() * 8, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_aval, av.data(), av.size() * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_pbterm, pbt.data(), pbt.size() * 8, hipMemcpyHostToDevice));
    return 0;
}

// loss / Σθ² scratch, per-net offsets and the last-block counter of
// mz_learner_grad_kernel
static int alloc_learner(mz_handle* h) {
    MZ_TRY(h, dalloc(h, &h->d_loss, 8));
    MZ_TRY(h, dalloc(h, &h->d_sq, 3 * MZ_L2_BLOCKS));
    size_t oc[6] = {h->flat_off[0], h->flat_off[1], h->flat_off[2], h->nparams[0], h->nparams[1], h->nparams[2]};
    MZ_TRY(h, dalloc(h, &h->d_netoff, 6));
    MZ_TRY(h, dalloc(h, &h->d_counter, 1));
    MZ_TRY(h, hipMemset(h->d_counter, 0, 4));
    MZ_TRY(h, dalloc(h, &h->d_fault, 1));
    MZ_TRY(h, hipMemset(h->d_fault, 0, 4));
    // debug (tests/test_fault_gpu.py): MZ_DEBUG_SKIP_PUBLISH=1 at create makes
    // tile / sample 0 of the cross-workgroup hand-offs skip its publish, with a
    // 10 ms poll bound, so the reported fault can be tested
    if (std::getenv("MZ_DEBUG_SKIP_PUBLISH")) { h->dbg_skip = 0; h->poll_ticks = 1000000ull; }
    MZ_TRY(h, hipMemcpy(h->d_netoff, oc, sizeof(oc), hipMemcpyHostToDevice));
    return 0;
}

static size_t rsearch_root_lds(const mz_handle* h) {
    const int gw = h->A > 16 ? 32 : 16;     // softmax / noise staging [16][gw] x 2
    return (size_t)std::max(h->rplan[0].lds_floats, h->rplan[1].lds_floats) * 4 + (size_t)2 * 16 * gw * 4;
}

// The downsampler of Learning.jl:175-187 (op for op as oracle/mz_oracle.c
// onet_build_resnet with downsample, `size` read as conv_kernel_size):
// Conv(k, C => C, stride 2), 2 blocks, Conv(k, C => 2C, stride 2), 3 blocks,
// MeanPool((3,3), stride 2, pad 1), 3 blocks, MeanPool — then the tail
// Conv(k, 2C => nf) + BatchNorm + blocks is the RPlan of rconf.  Parameters
// (Flux.params order, first in the representation's flat vector): strided
// conv W, b; block conv W, b, β, γ.  Returns the parameter count.
static size_t ds_build(mz_handle* h, DsPlan& D) {
    const mz_config& c = h->conf;
    const int kw = h->rhp.conv_kernel_size[0], kh = h->rhp.conv_kernel_size[1];
    int C = c.observation_shape[2] * (c.stacked_observations + 1) + c.stacked_observations;
    int w = c.observation_shape[0], hh = c.observation_shape[1];
    std::memset(&D, 0, sizeof(D));
    D.in_feat = w * hh * C;
    size_t n = 0;
    int cur = -1;
    auto s2 = [](int x, int k) { return (x + 2 * (k / 2) - k) / 2 + 1; };
    auto conv = [&](int cin, int cout, int stride, int bn, int act) -> DsLayer& {
        DsLayer& L = D.L[D.n++];
        L.kind = DS_CONV; L.cin = cin; L.cout = cout; L.kw = kw; L.kh = kh; L.pw = kw / 2; L.ph = kh / 2;
        L.stride = stride; L.Wi = w; L.Hi = hh;
        L.Wo = stride == 2 ? s2(w, kw) : w; L.Ho = stride == 2 ? s2(hh, kh) : hh;
        L.act = act; L.bn = bn;
        L.woff = (int)n; n += (size_t)kw * kh * cin * cout;
        L.boff = (int)n; n += (size_t)cout;
        if (bn) { L.bnoff = (int)n; n += (size_t)2 * cout; }
        L.pn = (int)(n - (size_t)L.woff);
        D.w_floats = std::max(D.w_floats, kw * kh * cin * cout);
        w = L.Wo; hh = L.Ho;
        return L;
    };
    auto strided = [&](int cin, int cout) {
        DsLayer& L = conv(cin, cout, 2, 0, MZ_ACT_IDENTITY);
        L.in_buf = cur; L.out_buf = cur == 0 ? 1 : 0; cur = L.out_buf;
    };
    auto block = [&](int f) {
        DsLayer& a = conv(f, f, 1, 1, MZ_ACT_RELU);
        a.in_buf = cur; a.out_buf = 1 - cur;
        DsLayer& b = conv(f, f, 1, 1, MZ_ACT_RELU);
        b.in_buf = 1 - cur; b.out_buf = cur; b.res_add = 1; b.res_buf = cur;
    };
    auto pool = [&](int f) {
        DsLayer& L = D.L[D.n++];
        L.kind = DS_POOL; L.cin = f; L.cout = f; L.kw = 3; L.kh = 3; L.pw = 1; L.ph = 1; L.stride = 2;
        L.Wi = w; L.Hi = hh; L.Wo = s2(w, 3); L.Ho = s2(hh, 3); L.act = MZ_ACT_IDENTITY;
        L.in_buf = cur; L.out_buf = 1 - cur; cur = L.out_buf;
        w = L.Wo; hh = L.Ho;
    };
    strided(C, C);
    for (int i = 0; i < 2; ++i) block(C);
    strided(C, 2 * C);
    for (int i = 0; i < 3; ++i) block(2 * C);
    pool(2 * C);
    for (int i = 0; i < 3; ++i) block(2 * C);
    pool(2 * C);
    D.L[D.n - 1].out_buf = -1;                       // the last layer writes the output to HBM
    D.out_feat = w * hh * 2 * C;
    for (int i = 0; i < D.n; ++i) {
        const DsLayer& L = D.L[i];
        if (i > 0) D.buf_floats = std::max(D.buf_floats, L.cin * L.Wi * L.Hi);
        D.buf_floats = std::max(D.buf_floats, L.cout * L.Wo * L.Ho);
    }
    D.buf_floats = (D.buf_floats + 3) & ~3;
    D.w_floats = (D.w_floats + 3) & ~3;
    h->rconf = c;
    h->rconf.observation_shape[0] = w; h->rconf.observation_shape[1] = hh; h->rconf.observation_shape[2] = 2 * C;
    h->rconf.stacked_observations = 0;
    // LDS: buffer 0 | buffer 1 (from buf_floats; the staged observation for layer 0 when it fits, layer 0
    // writing buffer 0) | one conv's packed parameters | the generic conv's weights and tap tables
    for (int i = 0; i < D.n; ++i) D.pn_max = std::max(D.pn_max, D.L[i].pn);
    D.pn_max = (D.pn_max + 3) & ~3;
    const size_t gen = (size_t)D.pn_max + D.w_floats + 512;
    const size_t in4 = ((size_t)D.in_feat + 3) & ~(size_t)3;
    D.ptot = (int)(n - (size_t)D.L[0].woff);
    D.stage_in = D.L[0].kind == DS_CONV && D.L[0].in_buf < 0 && D.L[0].out_buf == 0 && D.in_feat % 4 == 0 &&
                 D.L[0].woff % 4 == 0 && (size_t)2 * D.buf_floats + D.ptot <= in4 &&
                 ((size_t)D.buf_floats + std::max<size_t>(D.buf_floats, in4) + gen) * 4 <= kLdsMax;
    D.lds_floats = (int)((size_t)D.buf_floats + (D.stage_in ? std::max<size_t>(D.buf_floats, in4) : D.buf_floats));
    h->ds_lds = ((size_t)D.lds_floats + gen) * 4;
    return n;
}

// run the downsampler over n items: x (in_feat, n) -> y (rin_feat, n); with
// per_step > 0 item i uses the parameters flat + (i / per_step)·nflat (the
// multi-step learner's per-step bank), else the engine's
// the flat bank's per-step stride (rlearner_multi): nflat rounded up to 4 floats, so the downsampler's
// float4 parameter staging (DsParams.per_step) reads 16-byte aligned rows
static size_t fbank_stride(const mz_handle* h) { return (h->nflat + 3) / 4 * 4; }
static int ds_launch(mz_handle* h, const float* x, float* y, int n, hipStream_t st, const float* flat = nullptr,
                     int per_step = 0) {
    DsParams Q;
    Q.n_items = n; Q.bn_s = h->bn_s; Q.plan = h->d_dsplan; Q.flat = h->d_flat; Q.x = x; Q.y = y;
    Q.stamps = nullptr;
    Q.per_step = per_step; Q.flat_stride = fbank_stride(h);
    if (flat) Q.flat = flat;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, 128)));
    Q.stamps = h->d_stamps;
#endif
    void* args[] = {&Q};
    MZ_TRY(h, hipLaunchKernel((const void*)mz_downsample_kernel, dim3(n), dim3(DS_THREADS), args, h->ds_lds, st));
    return 0;
}
static int ensure_dsb(mz_handle* h, int n) {
    if (n <= h->dsb_cap) return 0;
    if (h->d_dsb) { (void)hipFree(h->d_dsb); h->d_dsb = nullptr; }
    MZ_TRY(h, hipMalloc(&h->d_dsb, (size_t)n * h->rin_feat * 4));
    h->dsb_cap = n;
    return 0;
}
static size_t rsearch_nets_lds(const mz_handle* h) {
    return (size_t)std::max(h->rplan[1].lds_floats, h->rplan[2].lds_floats) * 4;
}

int mz_engine_create_resnet(const mz_config* conf, const mz_resnet_hp* hyper, int device, int max_games,
                            uint64_t rng_seed, mz_handle** out) {
    g_create_error.clear();
    if (!conf || !hyper || !out) { g_create_error = "null argument"; return -2; }
    *out = nullptr;
    mz_handle* h = new mz_handle();
    h->kind = 1; h->conf = *conf; h->rhp = *hyper; h->device = device; h->max_games = max_games;
    h->seed = rng_seed;
    auto bad = [&](const std::string& m) { g_create_error = m; delete h; return -2; };
    const mz_config& c = *conf;
    if (c.action_space_size < 1 || c.action_space_size > 32)
        return bad("action_space_size must be in 1..32 (16- or 32-lane select groups)");
    if (c.players < 1 || c.players > 2) return bad("players must be 1 or 2");
    if (c.num_iters < 1 || c.num_iters > 65000) return bad("num_iters out of range");
    if (hyper->conv_kernel_size[0] % 2 == 0 || hyper->conv_kernel_size[1] % 2 == 0 ||
        hyper->conv_kernel_size[0] > 15 || hyper->conv_kernel_size[1] > 15)
        return bad("conv_kernel_size must be odd and <= 15 (Learning.jl:164 asserts odd)");
    if (hyper->num_filters < 1 || hyper->num_blocks < 0 || hyper->width_hidden < 1) return bad("bad ResNetHP");
    if (max_games < 1) return bad("max_games must be >= 1");
    if (hipSetDevice(device) != hipSuccess) return bad("hipSetDevice failed (no GPU?)");
    const int W = c.observation_shape[0], Hh = c.observation_shape[1], C = c.observation_shape[2];
    h->obs_feat = W * Hh * (C * (c.stacked_observations + 1) + c.stacked_observations);
    h->rconf = c;
    h->A = c.action_space_size; h->S = c.num_iters;
    if (hyper->downsample) {
        h->ds = 1;
        h->ds_n = ds_build(h, h->dsplan);
        if (h->dsplan.L[0].kw * h->dsplan.L[0].kh * 2 * h->dsplan.L[0].cin > 256)
            return bad("downsampler: conv_kernel_size x 2C input channels exceeds 256 taps");
        if (h->ds_lds > kLdsMax) return bad("downsampler activations exceed the LDS");
    }
    const int rW = h->rconf.observation_shape[0], rH = h->rconf.observation_shape[1];
    h->rin_feat = h->ds ? h->dsplan.out_feat : h->obs_feat;
    h->plane = rW * rH;
    h->H = rW * rH * hyper->num_filters;
    std::vector<RSpec> sp[3];
    size_t off = 0;
    for (int n = 0; n < 3; ++n) {
        sp[n] = rn_specs(h->rconf, *hyper, n, &h->nparams[n]);
        h->flat_off[n] = off;
        if (n == MZ_NET_REPR) h->nparams[n] += h->ds_n;     // downsampler params first
        off += h->nparams[n];
    }
    h->nflat = off;
    // widest tile whose three plans fit the LDS
    for (int ng = 16; ng >= 1 && !h->rn_ng; ng /= 2) {
        int wi = 0;
        bool fits = true;
        for (int n = 0; n < 3; ++n)
            fits &= (size_t)rn_plan(h, sp[n], n, ng, h->flat_off[n] + (n == 0 ? h->ds_n : 0), wi,
                                    nullptr).lds_floats * 4 <= kLdsMax;
        if (fits) h->rn_ng = ng;
    }
    if (!h->rn_ng) return bad("ResNet activations exceed the LDS even for one game per tile");
    h->bn_s = sqrtf(1.0f + 1e-5f);
    int rc = 0;
#define CK(x) do { if ((rc = (x)) != 0) { g_create_error = h->err; mz_engine_destroy(h); return rc; } } while (0)
    CK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess ? 0 : fail(h, "hipStreamCreate"));
    std::vector<int> sw;
    int wi = 0;
    h->rplan.resize(3);
    for (int n = 0; n < 3; ++n) {
        {
            int wt = wi;
            const bool sep = (size_t)rn_plan(h, sp[n], n, h->rn_ng, 0, wt, nullptr, true).lds_floats * 4 <= kLdsMax;
            h->rplan[n] = rn_plan(h, sp[n], n, h->rn_ng, h->flat_off[n] + (n == 0 ? h->ds_n : 0), wi, &sw, sep);
        }
        CK(h->rplan[n].n < 0 ? fail(h, "ResNet plan: a k-blocked output buffer") : 0);
        h->rn_lds[n] = (size_t)h->rplan[n].lds_floats * 4;
    }
    for (int n = 1; n < 3; ++n)                          // mz_rsearch_nets has no k-table path (NOKK)
        for (int i = 0; i < h->rplan[n].n; ++i) {
            const RLayer& L = h->rplan[n].L[i];
            CK(L.kk > 1 ? fail(h, "ResNet plan: a prediction / dynamics kernel > 1x1") : 0);
            // and applies a tanh only where the read-out does (RAWTANH): on the outputs
            CK(L.act == MZ_ACT_TANH && L.out_off != h->rplan[n].out0_off &&
                       !(h->rplan[n].out1_n && L.out_off == h->rplan[n].out1_off)
                   ? fail(h, "ResNet plan: a tanh layer that is not an output") : 0);
        }
    h->packed_w_n = sw.size(); h->packed_b_n = 0;
    h->rn_dyn_split = (int)sp[MZ_NET_DYN].size();     // the reward head: the dynamics layers of chain 2
    for (size_t i = 0; i < sp[MZ_NET_DYN].size(); ++i)
        if (sp[MZ_NET_DYN][i].chain == 2) { h->rn_dyn_split = (int)i; break; }
    {   // learner chain tiles: MZ_RN_NG_LEARN (power of two), default 1 (tools/rn_learner_ab.sh)
        const char* e = std::getenv("MZ_RN_NG_LEARN");
        int ngl = e ? std::atoi(e) : 1;
        if (ngl < 1 || ngl > h->rn_ng || (ngl & (ngl - 1))) ngl = 1;
        h->rn_ng_l = ngl;
        int wl = 0;
        h->rplan_l.resize(3);
        for (int n = 0; n < 3; ++n) {
            int wt = wl;
            const bool sep = (size_t)rn_plan(h, sp[n], n, ngl, 0, wt, nullptr, true).lds_floats * 4 <= kLdsMax;
            h->rplan_l[n] = rn_plan(h, sp[n], n, ngl, h->flat_off[n] + (n == 0 ? h->ds_n : 0), wl, nullptr, sep,
                                    &h->rtab);
            CK(h->rplan_l[n].n < 0 ? fail(h, "ResNet plan: a k-blocked output buffer") : 0);
            h->rn_lds_l = std::max(h->rn_lds_l, (size_t)h->rplan_l[n].lds_floats * 4);
        }
        h->rd_nb = rd_chain_ok(h);
        h->rd_chain = h->rd_nb > 0 && !std::getenv("MZ_RN_NO_RD");
        h->rp_pred = rp_pred_ok(h) && !std::getenv("MZ_RN_NO_RD");
    }
    h->inv_tile.assign(h->nflat, -1);
    for (size_t i = 0; i < sw.size(); ++i) if (sw[i] >= 0) h->inv_tile[(size_t)sw[i]] = (int)i;
    h->inv_small.assign(h->nflat, -1);
    auto al = [&](auto** p, size_t n) -> int { MZ_TRY(h, dalloc(h, p, n)); return 0; };
    auto al_i = [&](int** p, const std::vector<int>& v) -> int {
        MZ_TRY(h, dalloc(h, p, v.size()));
        MZ_TRY(h, hipMemcpy(*p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        return 0;
    };
    CK(al_i(&h->d_srcW, sw));
    CK(al_i(&h->d_inv_tile, h->inv_tile));
    CK(al_i(&h->d_inv_small, h->inv_small));
    CK(al(&h->d_rplan, 3));
    CK(hipMemcpy(h->d_rplan, h->rplan.data(), 3 * sizeof(RPlan), hipMemcpyHostToDevice) == hipSuccess
           ? 0 : fail(h, "copy"));
    if (!h->rtab.empty()) CK(al_i(&h->d_rtab, h->rtab));
    CK(al(&h->d_rplan_l, 3));
    CK(hipMemcpy(h->d_rplan_l, h->rplan_l.data(), 3 * sizeof(RPlan), hipMemcpyHostToDevice) == hipSuccess
           ? 0 : fail(h, "copy"));
    CK(al(&h->d_flat, h->nflat));
    CK(al(&h->d_Wp, h->packed_w_n));
    if (h->rd_chain && h->rp_pred) {                // second image set of mz_runroll_fused_r's ADAM blocks
        CK(al(&h->d_Wp2, h->packed_w_n));
        CK(hipMemset(h->d_Wp2, 0, h->packed_w_n * 4) == hipSuccess ? 0 : fail(h, "memset"));
    }
    CK(hipMemset(h->d_flat, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(repack(h));
    CK(al(&h->d_m, h->nflat)); CK(al(&h->d_v, h->nflat)); CK(al(&h->d_grad, h->nflat));
    CK(hipMemset(h->d_m, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(hipMemset(h->d_v, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(alloc_learner(h));
    const size_t lmax = std::max(h->rn_lds[0], std::max(h->rn_lds[1], h->rn_lds[2]));
    CK(hipFuncSetAttribute((const void*)mz_rnet_forward_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lmax) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(rnet)"));
    CK(rsearch_root_lds(h) > kLdsMax ? fail(h, "ResNet root tile exceeds the LDS") : 0);
    CK(hipFuncSetAttribute((const void*)mz_rsearch_root, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)rsearch_root_lds(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(root)"));
    CK(hipFuncSetAttribute((const void*)mz_rsearch_root32, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)rsearch_root_lds(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(root32)"));
    if (h->ds) {
        CK(hipFuncSetAttribute((const void*)mz_downsample_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)h->ds_lds) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(downsample)"));
        CK(al(&h->d_dsplan, 1));
        CK(hipMemcpy(h->d_dsplan, &h->dsplan, sizeof(DsPlan), hipMemcpyHostToDevice) == hipSuccess
               ? 0 : fail(h, "copy"));
        CK(al(&h->d_dsout, (size_t)max_games * h->rin_feat));
    }
    CK(hipFuncSetAttribute((const void*)mz_runroll_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lmax) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(runroll)"));
    CK(hipFuncSetAttribute((const void*)mz_runroll_pred, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lmax) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(runroll_pred)"));
    for (const void* k : {(const void*)mz_runroll_pred_n, (const void*)mz_runroll_pred_n1,
                          (const void*)mz_runroll_chain1})
        CK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->rn_lds_l) == hipSuccess
               ? 0 : fail(h, "hipFuncSetAttribute(runroll narrow)"));
    CK(hipFuncSetAttribute((const void*)mz_runroll_chain, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)h->rn_lds_l) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(runroll_chain)"));
    if (h->rd_chain)
        CK(hipFuncSetAttribute(h->rd_nb == 3 ? (const void*)mz_runroll_chain_r3 : (const void*)mz_runroll_chain_r,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)rd_chain_lds(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(runroll_chain_r)"));
    if (h->rp_pred)
        CK(hipFuncSetAttribute((const void*)mz_runroll_pred_r, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)rp_pred_lds(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(runroll_pred_r)"));
    if (h->rd_chain && h->rp_pred)
        CK(hipFuncSetAttribute(h->rd_nb == 3 ? (const void*)mz_runroll_fused_r3 : (const void*)mz_runroll_fused_r,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)std::max(rd_chain_lds(h), rp_pred_lds(h))) == hipSuccess
               ? 0 : fail(h, "hipFuncSetAttribute(runroll_fused_r)"));
    CK(hipFuncSetAttribute((const void*)mz_rsearch_nets, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)rsearch_nets_lds(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(nets)"));
    // search buffers (trees and hidden states in HBM)
    {
        const size_t G = (size_t)max_games, S = (size_t)h->S, A = (size_t)h->A, H = (size_t)h->H;
        h->tree_game_bytes = tree_game_bytes(h->S, h->A);
        CK(alloc_search_tables(h));
        // +64: the tree step copies the to_play bytes as dwords (up to 3 bytes past them)
        CK(al(&h->d_tree, G * h->tree_game_bytes + 64));
        CK(al(&h->d_hid, G * (S + 1) * H));
        {
            const int gw = h->A > 16 ? 32 : 16;
            const RsTreeLds L = rs_tree_lds(h->S, h->tree_game_bytes, gw);
            h->rtree_lds = (size_t)L.total <= kLdsMax && !std::getenv("MZ_RTREE_HBM") ? (size_t)L.total : 0;
            if (h->rtree_lds)
                CK(hipFuncSetAttribute(gw == 32 ? (const void*)mz_rsearch_tree_lds32 : (const void*)mz_rsearch_tree_lds,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->rtree_lds) == hipSuccess
                       ? 0 : fail(h, "hipFuncSetAttribute(tree_lds)"));
        }
        CK(al(&h->d_rpath, G * 2 * (S + 2))); CK(al(&h->d_rgst, G * RG_INTS));
        CK(al(&h->d_rcache, G * (S + 1))); CK(al(&h->d_rnN, G * (S + 1)));
        CK(al(&h->d_rhk, G * (S + 1))); CK(al(&h->d_rov, G)); CK(al(&h->d_rologit, G * A)); CK(al(&h->d_ror, G));
        CK(al(&h->d_obs, G * h->obs_feat)); CK(al(&h->d_legal, G * A)); CK(al(&h->d_tp, G));
        CK(al(&h->d_cv, G * A)); CK(al(&h->d_rv, G)); CK(al(&h->d_act, G));
    }
    CK(hipStreamSynchronize(h->stream) == hipSuccess ? 0 : fail(h, "sync"));
#undef CK
    *out = h;
    return 0;
}

// ---- RCCL, loaded on first use (dlopen: libmz has no link dependency on it;
// RTLD_NOLOAD first so a process that already holds an RCCL — torch's — shares it)
// ncclUniqueId: a 128-byte struct that ncclCommInitRank takes BY VALUE
struct RcclId { uint8_t b[MZ_DP_ID_BYTES]; };
struct RcclApi {
    bool ok = false;
    int (*get_id)(void*) = nullptr;                                    // ncclGetUniqueId(ncclUniqueId*)
    int (*init_rank)(void**, int, RcclId, int) = nullptr;              // ncclCommInitRank(comm*, n, id, rank)
    int (*allreduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*destroy)(void*) = nullptr;
    const char* (*err)(int) = nullptr;
};
static RcclApi& rccl() {
    static RcclApi api;
    static bool tried = false;
    if (tried) return api;
    tried = true;
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW);
    if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!lib) return api;
    api.get_id = reinterpret_cast<int (*)(void*)>(dlsym(lib, "ncclGetUniqueId"));
    api.allreduce = reinterpret_cast<int (*)(const void*, void*, size_t, int, int, void*, hipStream_t)>(
        dlsym(lib, "ncclAllReduce"));
    api.destroy = reinterpret_cast<int (*)(void*)>(dlsym(lib, "ncclCommDestroy"));
    api.err = reinterpret_cast<const char* (*)(int)>(dlsym(lib, "ncclGetErrorString"));
    api.init_rank = reinterpret_cast<int (*)(void**, int, RcclId, int)>(dlsym(lib, "ncclCommInitRank"));
    api.ok = api.get_id && api.init_rank && api.allreduce && api.destroy;
    return api;
}
static void dp_destroy(mz_handle* h) {
    if (h->dp_comm && rccl().ok) (void)rccl().destroy(h->dp_comm);
    h->dp_comm = nullptr; h->dp_world = 0;
}

void mz_engine_destroy(mz_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (hipEvent_t e : h->tev) (void)hipEventDestroy(e);
    for (void* p : h->allocs) (void)hipFree(p);
    for (void* p : h->sp_allocs) (void)hipFree(p);
    if (h->d_dsb) (void)hipFree(h->d_dsb);
    if (h->h_tr_cnt) (void)hipHostFree(h->h_tr_cnt);
    if (h->h_tr_pub) (void)hipHostFree(h->h_tr_pub);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    dp_destroy(h);
    delete h;
}

int mz_engine_create(const mz_config* conf, const mz_ffhp* hyper, int device, int max_games, uint64_t rng_seed,
                     mz_handle** out) {
    g_create_error.clear();
    if (!conf || !hyper || !out) { g_create_error = "null argument"; return -2; }
    *out = nullptr;
    mz_handle* h = new mz_handle();
    h->conf = *conf; h->hp = *hyper; h->device = device; h->max_games = max_games; h->seed = rng_seed;
    auto bad = [&](const std::string& m) { g_create_error = m; delete h; return -2; };
    const mz_config& c = *conf;
    if (c.action_space_size < 1 || c.action_space_size > 16)
        return bad("action_space_size must be in 1..16 (16-lane select groups)");
    if (c.players < 1 || c.players > 2) return bad("players must be 1 or 2");
    if (c.num_iters < 1 || c.num_iters >= (1 << 20)) return bad("num_iters out of range");
    if (hyper->hidden_state_size != c.observation_shape[0] * c.observation_shape[1] * c.observation_shape[2])
        return bad("hidden_state_size must equal prod(observation_shape) (the FC path reshapes h to it)");
    if (max_games < 1) return bad("max_games must be >= 1");
    if (hipSetDevice(device) != hipSuccess) return bad("hipSetDevice failed (no GPU?)");
    build_specs(h);
    if (c.num_iters > 65000) return bad("num_iters must be <= 65000 (16-bit visit counts in the tree)");
    h->tree_game_bytes = tree_game_bytes(c.num_iters, c.action_space_size);
    h->lds_tree = search_lds_base(h) + (size_t)MZ_TILE * h->tree_game_bytes <= kLdsMax;
    if (search_lds_bytes(h) > kLdsMax) return bad("LDS budget exceeded (width/num_iters too large)");
    int rc = 0;
#define CK(x) do { if ((rc = (x)) != 0) { g_create_error = h->err; mz_engine_destroy(h); return rc; } } while (0)
    CK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess ? 0 : fail(h, "hipStreamCreate"));
    CK(build_plans(h));
    CK(build_pack_index(h));
    auto al_i = [&](int** p, const std::vector<int>& v) -> int {
        MZ_TRY(h, dalloc(h, p, v.size()));
        MZ_TRY(h, hipMemcpy(*p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        return 0;
    };
    {
        int r = build_small(h);
        if (r < 0) { g_create_error = h->err; mz_engine_destroy(h); return r; }
        h->small_ok = r == 1;
        for (int ti = 0; ti < 3 && h->small_ok; ++ti) h->small_ok = h->sm_lds[ti] <= kLdsMax;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->n_cu = prop.multiProcessorCount;
        if (!h->small_ok) h->inv_small.assign(h->nflat, -1);
        CK(al_i(&h->d_inv_tile, h->inv_tile));
        CK(al_i(&h->d_inv_small, h->inv_small));
        const char* fk = std::getenv("MZ_SEARCH_KERNEL");
        if (fk) h->force_kernel = std::strcmp(fk, "tile16") == 0 ? 1 : std::strcmp(fk, "small") == 0 ? 2 : 0;
        const char* ft = std::getenv("MZ_SMALL_T");
        if (ft) { const int t = std::atoi(ft); h->force_T = (t == 1 || t == 2 || t == 4) ? t : 0; }
        if (h->small_ok) {
            const void* ks[6] = {(const void*)mz_search_small1, (const void*)mz_search_small2,
                                 (const void*)mz_search_small4, (const void*)mz_search_small1_bn,
                                 (const void*)mz_search_small2_bn, (const void*)mz_search_small4_bn};
            for (int ti = 0; ti < 6; ++ti)
                CK(hipFuncSetAttribute(ks[ti], hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->sm_lds[ti % 3]) ==
                           hipSuccess ? 0 : fail(h, "hipFuncSetAttribute(small)"));
            const void* ku[4] = {(const void*)mz_unroll_small1, (const void*)mz_unroll_small2,
                                 (const void*)mz_unroll_small1_bn, (const void*)mz_unroll_small2_bn};
            for (int ti = 0; ti < 4; ++ti)
                CK(hipFuncSetAttribute(ku[ti], hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)unroll_small_lds(h, ti & 1)) == hipSuccess
                       ? 0 : fail(h, "hipFuncSetAttribute(unroll_small)"));
        }
    }
    const int S = h->S, A = h->A, H = h->H;
    const size_t G = (size_t)max_games;
    auto al = [&](auto** p, size_t n) -> int { MZ_TRY(h, dalloc(h, p, n)); return 0; };
    CK(al(&h->d_flat, h->nflat));
    CK(al(&h->d_Wp, h->packed_w_n));
    CK(al(&h->d_Bp, h->packed_b_n));
    if (h->small_ok) {
        CK(al(&h->d_Wp2, h->packed_w_n)); CK(al(&h->d_Bp2, h->packed_b_n));
        CK(al(&h->d_sm_w2, h->sm_w_n)); CK(al(&h->d_sm_bias2, h->sm_b_n));
        const void* kl[8] = {(const void*)mz_learn_small1, (const void*)mz_learn_small2,
                             (const void*)mz_learn_multi1, (const void*)mz_learn_multi2,
                             (const void*)mz_learn_small1_bn, (const void*)mz_learn_small2_bn,
                             (const void*)mz_learn_multi1_bn, (const void*)mz_learn_multi2_bn};
        for (int ti = 0; ti < 8; ++ti)
            CK(hipFuncSetAttribute(kl[ti], hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)unroll_small_lds(h, ti & 1)) == hipSuccess
                   ? 0 : fail(h, "hipFuncSetAttribute(learn_small)"));
        const void* k4[2] = {(const void*)mz_learn_multi4, (const void*)mz_learn_multi4_bn};
        for (int j = 0; j < 2; ++j)
            CK(hipFuncSetAttribute(k4[j], hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)unroll_small_lds(h, 2)) == hipSuccess
                   ? 0 : fail(h, "hipFuncSetAttribute(learn_multi4)"));
    }
    CK(hipMemset(h->d_flat, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(repack(h));
    // tables: libm log2/sqrt on the host, the values the oracle computes inline
    std::vector<double> pbc(S + 2), sq(S + 2);
    for (int n = 0; n < S + 2; ++n) {
        pbc[n] = std::log2((double)(n + c.pb_c_base + 1) / (double)c.pb_c_base) + (double)c.pb_c_init;
        sq[n] = std::sqrt((double)n);
    }
    std::vector<float> av(A);
    for (int a = 0; a < A; ++a) av[a] = (float)((double)(a + 1) / (double)A);
    CK(al(&h->d_pbc, pbc.size()));
    CK(al(&h->d_sqrt, sq.size()));
    CK(al(&h->d_aval, av.size()));
    CK(hipMemcpy(h->d_pbc, pbc.data(), pbc.size() * 8, hipMemcpyHostToDevice) == hipSuccess ? 0 : fail(h, "copy"));
    CK(hipMemcpy(h->d_sqrt, sq.data(), sq.size() * 8, hipMemcpyHostToDevice) == hipSuccess ? 0 : fail(h, "copy"));
    CK(hipMemcpy(h->d_aval, av.data(), av.size() * 4, hipMemcpyHostToDevice) == hipSuccess ? 0 : fail(h, "copy"));
    // the same f64 expression select evaluates, tabulated (Nc < Np <= S+1)
    std::vector<double> pbt(pbterm_count(S), 0.0);
    for (int np = 0; np <= S + 1; ++np)
        for (int nc = 0; nc <= np; ++nc) pbt[pbterm_index(np, nc)] = pbc[np] * (sq[np] / (double)(nc + 1));
    CK(al(&h->d_pbterm, pbt.size()));
    CK(hipMemcpy(h->d_pbterm, pbt.data(), pbt.size() * 8, hipMemcpyHostToDevice) == hipSuccess ? 0 : fail(h, "copy"));
    CK(al(&h->d_tree, G * h->tree_game_bytes));
    CK(al(&h->d_hid, G * (S + 1) * H));
    CK(al(&h->d_obs, G * h->obs_feat)); CK(al(&h->d_legal, G * A)); CK(al(&h->d_tp, G));
    CK(al(&h->d_cv, G * A)); CK(al(&h->d_rv, G)); CK(al(&h->d_act, G));
    CK(al(&h->d_m, h->nflat)); CK(al(&h->d_v, h->nflat)); CK(al(&h->d_grad, h->nflat));
    CK(hipMemset(h->d_m, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(hipMemset(h->d_v, 0, h->nflat * 4) == hipSuccess ? 0 : fail(h, "memset"));
    CK(alloc_learner(h));
    h->use_res = h->d_plan_sim_res != nullptr && std::getenv("MZ_NO_RESIDENT") == nullptr;
    {
        const search_fn ks[4] = {mz_search_kernel_lds, mz_search_kernel_hbm, mz_search_kernel_lds_res,
                                 mz_search_kernel_hbm_res};
        for (auto k : ks)
            CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)search_lds_bytes(h)) == hipSuccess ? 0 : fail(h, "hipFuncSetAttribute"));
    }
    CK(hipStreamSynchronize(h->stream) == hipSuccess ? 0 : fail(h, "sync"));
#undef CK
    *out = h;
    return 0;
}

int mz_net_param_count(const mz_handle* h, int net, size_t* n) {
    if (!h || !n || net < 0 || net > 2) return -2;
    *n = h->nparams[net];
    return 0;
}

int mz_grad_count(const mz_handle* h, size_t* n) {
    if (!h || !n) return -2;
    *n = h->nflat;
    return 0;
}

int mz_weights_set(mz_handle* h, int net, const float* flat, size_t n) {
    if (!h) return -2;
    if (net < 0 || net > 2) return fail(h, "bad net id");
    if (n != h->nparams[net]) return fail(h, "weights_set: wrong parameter count");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);                  // no search / learner launch still reads the old weights
    MZ_TRY(h, hipMemcpyAsync(h->d_flat + h->flat_off[net], flat, n * 4, hipMemcpyHostToDevice, h->stream));
    if (repack(h)) return -1;
    MZ_SYNC(h);
    return 0;
}

int mz_weights_get(mz_handle* h, int net, float* flat, size_t n) {
    if (!h) return -2;
    if (net < 0 || net > 2) return fail(h, "bad net id");
    if (n != h->nparams[net]) return fail(h, "weights_get: wrong parameter count");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);                  // learner steps queued on any stream have landed
    MZ_TRY(h, hipMemcpyAsync(flat, h->d_flat + h->flat_off[net], n * 4, hipMemcpyDeviceToHost, h->stream));
    MZ_SYNC(h);
    return 0;
}

static int rnet_forward(mz_handle* h, int net, const float* x, int n, float* out0, float* out1) {
    const RPlan& R = h->rplan[net];
    const bool ds = h->ds && net == MZ_NET_REPR;
    const int xin = ds ? h->obs_feat : R.in_feat;     // the raw observation goes through the downsampler
    float *dx = nullptr, *d0 = nullptr, *d1 = nullptr;
    MZ_TRY(h, hipMalloc(&dx, (size_t)n * xin * 4));
    MZ_TRY(h, hipMalloc(&d0, (size_t)n * R.out0_n * 4));
    MZ_TRY(h, hipMalloc(&d1, (size_t)n * std::max(R.out1_n, 1) * 4));
    (void)hipMemcpyAsync(dx, x, (size_t)n * xin * 4, hipMemcpyHostToDevice, h->stream);
    if (ds) {
        if (ensure_dsb(h, n) || ds_launch(h, dx, h->d_dsb, n, h->stream)) {
            (void)hipFree(dx); (void)hipFree(d0); (void)hipFree(d1);
            return -1;
        }
    }
    RNetParams Q;
    Q.ng = h->rn_ng; Q.W = h->rconf.observation_shape[0]; Q.H = h->rconf.observation_shape[1];
    Q.P = Q.W * Q.H; Q.n_items = n; Q.softmax1 = net == MZ_NET_PRED; Q.bn_s = h->bn_s;
    Q.plan = h->d_rplan + net; Q.Wimg = h->d_Wp; Q.flat = h->d_flat; Q.x = ds ? h->d_dsb : dx; Q.out0 = d0;
    Q.out1 = d1;
    void* args[] = {&Q};
    hipError_t le = hipLaunchKernel((const void*)mz_rnet_forward_kernel, dim3((n + Q.ng - 1) / Q.ng), dim3(RN_THREADS),
                                    args, h->rn_lds[net], h->stream);
    (void)hipMemcpyAsync(out0, d0, (size_t)n * R.out0_n * 4, hipMemcpyDeviceToHost, h->stream);
    if (out1 && R.out1_n) (void)hipMemcpyAsync(out1, d1, (size_t)n * R.out1_n * 4, hipMemcpyDeviceToHost, h->stream);
    hipError_t se = sync_device(h);
    (void)hipFree(dx); (void)hipFree(d0); (void)hipFree(d1);
    MZ_TRY(h, le);
    MZ_TRY(h, se);
    return check_fault(h);
}

int mz_net_forward(mz_handle* h, int net, const float* x, int n, float* out0, float* out1) {
    if (!h) return -2;
    if (net < 0 || net > 2) return fail(h, "bad net id");
    if (n < 0) return fail(h, "negative batch");
    if (n == 0) return 0;
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);                  // weights written by `_dev` calls on other streams
    if (h->kind == 1) return rnet_forward(h, net, x, n, out0, out1);
    const int H = h->H, A = h->A;
    const int in_feat = net == MZ_NET_REPR ? h->obs_feat : net == MZ_NET_PRED ? H : H + h->plane;
    const int in_off = net == MZ_NET_REPR ? h->lay.x_rep : net == MZ_NET_PRED ? h->lay.x_pred : h->lay.x_dyn;
    const int o0 = net == MZ_NET_PRED ? 1 : H;
    const int o0_off = net == MZ_NET_PRED ? h->lay.v_out : h->lay.h_out;
    const int o1 = net == MZ_NET_PRED ? A : 1;
    const int o1_off = net == MZ_NET_PRED ? h->lay.p_out : h->lay.r_out;
    float *dx = nullptr, *d0 = nullptr, *d1 = nullptr;
    MZ_TRY(h, hipMalloc(&dx, (size_t)n * in_feat * 4));
    MZ_TRY(h, hipMalloc(&d0, (size_t)n * o0 * 4));
    MZ_TRY(h, hipMalloc(&d1, (size_t)n * o1 * 4));
    (void)hipMemcpyAsync(dx, x, (size_t)n * in_feat * 4, hipMemcpyHostToDevice, h->stream);
    hipLaunchKernelGGL(mz_forward_kernel, dim3((n + MZ_TILE - 1) / MZ_TILE), dim3(MZ_THREADS),
                       (size_t)h->lay.total * 4, h->stream, h->d_plan[net], h->d_Wp, h->d_Bp, h->lay.total, in_off,
                       in_feat, dx, n, o0_off, o0, d0, o1_off, o1, net == MZ_NET_REPR ? nullptr : d1,
                       net == MZ_NET_PRED ? 1 : 0, net == MZ_NET_PRED ? h->lay.v_act : MZ_ACT_IDENTITY,
                       net == MZ_NET_DYN ? h->lay.r_act : MZ_ACT_IDENTITY);
    hipError_t le = hipGetLastError();
    (void)hipMemcpyAsync(out0, d0, (size_t)n * o0 * 4, hipMemcpyDeviceToHost, h->stream);
    if (out1 && net != MZ_NET_REPR) (void)hipMemcpyAsync(out1, d1, (size_t)n * o1 * 4, hipMemcpyDeviceToHost, h->stream);
    hipError_t se = sync_device(h);
    (void)hipFree(dx); (void)hipFree(d0); (void)hipFree(d1);
    MZ_TRY(h, le);
    MZ_TRY(h, se);
    return check_fault(h);
}

// ResNet search: root launch, S x (tree step, networks), final tree step
static int rsearch(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask, const int32_t* to_play,
                   int exploration, uint32_t rng_step, uint32_t game_offset, float temperature, float* child_visits,
                   float* root_value, int32_t* action_out, hipStream_t st, const float* temp_g) {
    RSearchParams P;
    std::memset(&P, 0, sizeof(P));
    P.temp_g = temp_g;
    P.G = G; P.S = h->S; P.A = h->A; P.H = h->H; P.W = h->rconf.observation_shape[0];
    P.P = h->plane; P.players = h->conf.players; P.obs_feat = h->rin_feat; P.exploration = exploration;
    P.rng_step = rng_step; P.game_offset = game_offset; P.seed = h->seed; P.temperature = temperature;
    P.discount = h->conf.discount; P.dirichlet_alpha = h->conf.dirichlet_alpha;
    P.exploration_eps = h->conf.exploration_eps;
    P.obs = obs; P.legal = legal_mask; P.to_play = to_play;
    P.child_visits = child_visits; P.root_value = root_value; P.action_out = action_out;
    P.pbc_tab = h->d_pbc; P.sqrt_tab = h->d_sqrt; P.aval_tab = h->d_aval; P.pbterm = h->d_pbterm;
    P.tree = h->d_tree; P.tree_game_bytes = h->tree_game_bytes; P.hid = h->d_hid;
    P.cache = h->d_rcache; P.nN = h->d_rnN;
    P.path = h->d_rpath; P.gst = h->d_rgst; P.hk = h->d_rhk;
    P.o_v = h->d_rov; P.o_logit = h->d_rologit; P.o_r = h->d_ror;
    P.ng = h->rn_ng; P.bn_s = h->bn_s; P.plans = h->d_rplan; P.Wimg = h->d_Wp; P.flat = h->d_flat;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, 128)));
    P.stamps = h->d_stamps;
#endif
    if (h->ds) {                                    // representation: downsampler, then the tail in the root
        if (ds_launch(h, obs, h->d_dsout, G, st)) return -1;
        P.obs = h->d_dsout;
    }
    void* args[] = {&P};
    const int gw = h->A > 16 ? 32 : 16;             // lanes per game in the tree kernels
    const unsigned tiles = (unsigned)((G + P.ng - 1) / P.ng), groups = (unsigned)((G + 256 / gw - 1) / (256 / gw));
    // the dynamics reward head on the prediction workgroup (RSearchParams.rew_split)
    static const bool no_rsplit = std::getenv("MZ_RN_NO_RSPLIT") != nullptr;
    if (!no_rsplit && !h->d_rtrunk) {
        const size_t mt = (size_t)(h->max_games + P.ng - 1) / P.ng;
        MZ_TRY(h, dalloc(h, &h->d_rtrunk, (size_t)h->max_games * h->H));
        MZ_TRY(h, dalloc(h, &h->d_tprog, mt));
        MZ_TRY(h, hipMemset(h->d_tprog, 0, mt * sizeof(unsigned long long)));
    }
    P.rew_split = no_rsplit ? 0 : 1;
    P.trunk_nl = 1 + 2 * h->rhp.num_blocks; P.dyn_split = h->rn_dyn_split;
    P.trunk = h->d_rtrunk; P.tprog = h->d_tprog;
    P.fault = h->d_fault; P.poll_ticks = h->poll_ticks; P.dbg_skip = h->dbg_skip;
    static const bool no_moved_skip = std::getenv("MZ_NO_MOVED_SKIP") != nullptr;   // A/B only
    P.no_moved_skip = no_moved_skip ? 1 : 0;
    const void* kroot = gw == 32 ? (const void*)mz_rsearch_root32 : (const void*)mz_rsearch_root;
    // tree step: LDS-cached (one wave per 64/gw games) unless the tree exceeds the LDS
    const bool tl = h->rtree_lds != 0;
    const void* ktree = tl ? (gw == 32 ? (const void*)mz_rsearch_tree_lds32 : (const void*)mz_rsearch_tree_lds)
                           : (gw == 32 ? (const void*)mz_rsearch_tree32 : (const void*)mz_rsearch_tree);
    const unsigned tgrid = tl ? (unsigned)((G + 64 / gw - 1) / (64 / gw)) : groups;
    MZ_TRY(h, hipLaunchKernel(kroot, dim3(tiles), dim3(RN_THREADS), args, rsearch_root_lds(h), st));
    for (int s = 0; s <= h->S; ++s) {
        P.s = s;
        MZ_TRY(h, hipLaunchKernel(ktree, dim3(tgrid), dim3(tl ? 64 * RT_WAVES : 256), args, tl ? h->rtree_lds : 0, st));
        if (s == h->S) break;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (h->time_nets) {
            if (h->tev_used + 2 > h->tev.size())
                for (int i = 0; i < 2; ++i) {
                    hipEvent_t e;
                    MZ_TRY(h, hipEventCreate(&e));
                    h->tev.push_back(e);
                }
            e0 = h->tev[h->tev_used++]; e1 = h->tev[h->tev_used++];
            MZ_TRY(h, hipEventRecord(e0, st));
        }
        P.tepoch = ++h->tprog_epoch;
        MZ_TRY(h, hipLaunchKernel((const void*)mz_rsearch_nets, dim3(tiles, 2), dim3(RN_THREADS_NETS), args,
                                  rsearch_nets_lds(h), st));
        if (e1) MZ_TRY(h, hipEventRecord(e1, st));
    }
    h->last_variant = "mz_rsearch";
    return 0;
}

// the batched search; temp_g: per-game temperatures (device, G) or NULL =
// `temperature` for every game
static int search_dev(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask, const int32_t* to_play,
                      int exploration, uint32_t rng_step, uint32_t game_offset, float temperature,
                      float* child_visits, float* root_value, int32_t* action_out, void* stream,
                      const float* temp_g) {
    if (!h) return -2;
    if (G < 0 || G > h->max_games) return fail(h, "G exceeds max_games");
    if (G == 0) return 0;
    if (h->kind == 1)
        return rsearch(h, G, obs, legal_mask, to_play, exploration, rng_step, game_offset, temperature,
                       child_visits, root_value, action_out, stream ? (hipStream_t)stream : h->stream, temp_g);
    SearchParams P;
    std::memset(&P, 0, sizeof(P));
    P.temp_g = temp_g;
    P.G = G; P.S = h->S; P.A = h->A; P.H = h->H; P.players = h->conf.players; P.obs_feat = h->obs_feat;
    P.plane = h->plane; P.exploration = exploration; P.rng_step = rng_step; P.game_offset = game_offset;
    P.seed = h->seed; P.temperature = temperature; P.discount = h->conf.discount;
    P.dirichlet_alpha = h->conf.dirichlet_alpha; P.exploration_eps = h->conf.exploration_eps;
    P.obs = obs; P.legal = legal_mask; P.to_play = to_play;
    P.child_visits = child_visits; P.root_value = root_value; P.action_out = action_out;
    P.Wp = h->d_Wp; P.Bp = h->d_Bp; P.plan_root = h->d_plan[3]; P.plan_sim = h->d_plan[4];
    P.plan_sim_res = h->use_res ? h->d_plan_sim_res : nullptr;
    P.lay = h->lay; P.pbc_tab = h->d_pbc; P.sqrt_tab = h->d_sqrt; P.aval_tab = h->d_aval;
    P.tree = h->d_tree; P.tree_game_bytes = h->tree_game_bytes; P.dump_tree = h->dump_tree;
    P.hid = h->d_hid;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * h->max_games));
    P.stamps = h->d_stamps;
#endif
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const bool small = h->small_ok && h->force_kernel != 1 && (h->force_kernel == 2 || G <= 4 * h->n_cu);
    if (small) {
        const int T = h->force_T ? h->force_T : G <= h->n_cu ? 1 : G <= 2 * h->n_cu ? 2 : 4;
        const int ti = T == 1 ? 0 : T == 2 ? 1 : 2;
        SmallParams Q;
        std::memset(&Q, 0, sizeof(Q));
        Q.temp_g = temp_g;
        Q.G = G; Q.S = h->S; Q.A = h->A; Q.H = h->H; Q.players = h->conf.players; Q.obs_feat = h->obs_feat;
        Q.plane = h->plane; Q.exploration = exploration; Q.rng_step = rng_step; Q.game_offset = game_offset;
        Q.seed = h->seed; Q.temperature = temperature; Q.discount = h->conf.discount;
        Q.dirichlet_alpha = h->conf.dirichlet_alpha; Q.exploration_eps = h->conf.exploration_eps;
        Q.obs = obs; Q.legal = legal_mask; Q.to_play = to_play;
        Q.child_visits = child_visits; Q.root_value = root_value; Q.action_out = action_out;
        Q.n_sim = h->sm_n_sim; Q.n_root = h->sm_n_root;
        Q.w_sim = h->d_sm_w;
        std::memcpy(Q.nzm, h->sm_nzm.data(), sizeof(Q.nzm));
        Q.bn = h->sm_bn;
        Q.zero16 = reinterpret_cast<const float4*>(h->d_zero16);
        Q.w_root = h->d_sm_w + (size_t)h->sm_n_sim * SM_SLOTS * 256 * 16;
        Q.rec = h->d_sm_rec[ti]; Q.bias = h->d_sm_bias;
        const int* lay = h->sm_lay[ti];
        Q.act_total = lay[0]; Q.x_rep = lay[1]; Q.x_pred = lay[2]; Q.x_dyn = lay[3]; Q.h_out = lay[4];
        Q.v_out = lay[5]; Q.p_out = lay[6]; Q.r_out = lay[7];
        Q.v_act = h->lay.v_act; Q.r_act = h->lay.r_act;
        Q.pbc_tab = h->d_pbc; Q.sqrt_tab = h->d_sqrt; Q.aval_tab = h->d_aval;
        Q.pbterm = h->d_pbterm;
        Q.tree = h->d_tree; Q.tree_game_bytes = h->tree_game_bytes; Q.dump_tree = h->dump_tree;
#ifdef MZ_STAMPS
        Q.stamps = h->d_stamps;
#endif
        const void* k = h->sm_bn ? (T == 1 ? (const void*)mz_search_small1_bn : T == 2 ? (const void*)mz_search_small2_bn
                                                                                   : (const void*)mz_search_small4_bn)
                                 : (T == 1 ? (const void*)mz_search_small1 : T == 2 ? (const void*)mz_search_small2
                                                                                   : (const void*)mz_search_small4);
        void* args[] = {&Q};
        MZ_TRY(h, hipLaunchKernel(k, dim3((G + T - 1) / T), dim3(SM_THREADS), args, h->sm_lds[ti], st));
        h->last_variant = std::string(T == 1 ? "mz_search_small1" : T == 2 ? "mz_search_small2" : "mz_search_small4") +
                          (h->sm_bn ? "_bn" : "");
    } else {
        hipLaunchKernelGGL(search_kernel(h), dim3((G + MZ_TILE - 1) / MZ_TILE), dim3(MZ_THREADS),
                           search_lds_bytes(h), st, P);
        h->last_variant = h->use_res ? (h->lds_tree ? "mz_search_kernel_lds_res" : "mz_search_kernel_hbm_res")
                                     : (h->lds_tree ? "mz_search_kernel_lds" : "mz_search_kernel_hbm");
    }
    MZ_TRY(h, hipGetLastError());
    return 0;
}

int mz_mcts_search_dev(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask, const int32_t* to_play,
                       int exploration, uint32_t rng_step, uint32_t game_offset, float temperature,
                       float* child_visits, float* root_value, int32_t* action_out, void* stream) {
    return search_dev(h, G, obs, legal_mask, to_play, exploration, rng_step, game_offset, temperature, child_visits,
                      root_value, action_out, stream, nullptr);
}

int mz_mcts_search(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask, const int32_t* to_play,
                   int exploration, uint32_t rng_step, uint32_t game_offset, float temperature, float* child_visits,
                   float* root_value, int32_t* action_out) {
    if (!h) return -2;
    if (G < 0 || G > h->max_games) return fail(h, "G exceeds max_games");
    if (G == 0) return 0;
    const int A = h->A;
    for (int g = 0; g < G; ++g) {       // @assert !isempty(legal_actions) (SelfPlay.jl:243)
        int any = 0;
        for (int a = 0; a < A; ++a) any |= legal_mask[(size_t)g * A + a] != 0;
        if (!any) return fail(h, "Legal actions should not be an empty array (game " + std::to_string(g) + ")");
        if (to_play[g] < 1 || to_play[g] > h->conf.players) return fail(h, "to_play out of range");
    }
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);                  // `_dev` work on other streams first
    MZ_TRY(h, hipMemcpyAsync(h->d_obs, obs, (size_t)G * h->obs_feat * 4, hipMemcpyHostToDevice, h->stream));
    MZ_TRY(h, hipMemcpyAsync(h->d_legal, legal_mask, (size_t)G * A, hipMemcpyHostToDevice, h->stream));
    MZ_TRY(h, hipMemcpyAsync(h->d_tp, to_play, (size_t)G * 4, hipMemcpyHostToDevice, h->stream));
    int rc = mz_mcts_search_dev(h, G, h->d_obs, h->d_legal, h->d_tp, exploration, rng_step, game_offset, temperature,
                                h->d_cv, h->d_rv, h->d_act, h->stream);
    if (rc) return rc;
    MZ_TRY(h, hipMemcpyAsync(child_visits, h->d_cv, (size_t)G * A * 4, hipMemcpyDeviceToHost, h->stream));
    MZ_TRY(h, hipMemcpyAsync(root_value, h->d_rv, (size_t)G * 4, hipMemcpyDeviceToHost, h->stream));
    MZ_TRY(h, hipMemcpyAsync(action_out, h->d_act, (size_t)G * 4, hipMemcpyDeviceToHost, h->stream));
    MZ_SYNC(h);
    return 0;
}

int mz_set_sync_stream(mz_handle* h, void* stream, int narrow) {
    if (!h) return -1;
    h->sync_stream = (hipStream_t)stream;
    h->sync_narrow = narrow != 0;
    return 0;
}

int mz_debug_enable(mz_handle* h, int flags) {
    if (!h) return -2;
    h->dump_tree = flags & 1;
    h->time_nets = (flags >> 1) & 1;
    h->time_unroll = (flags >> 2) & 1;
    return 0;
}

int mz_debug_tree(mz_handle* h, int G, int32_t* eN, float* eW, float* eP, float* eR, int32_t* eC, int32_t* ntp) {
    if (!h) return -2;
    if (G < 0 || G > h->max_games) return fail(h, "G exceeds max_games");
    if (h->lds_tree && !h->dump_tree) return fail(h, "mz_debug_tree needs mz_debug_enable(h, 1) before the search");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    const int S = h->S, A = h->A, NN = S + 1, E = NN * A;
    const size_t gb = h->tree_game_bytes;
    std::vector<char> buf((size_t)G * gb);
    MZ_TRY(h, hipMemcpy(buf.data(), h->d_tree, buf.size(), hipMemcpyDeviceToHost));
    for (int g = 0; g < G; ++g) {
        const char* b = buf.data() + (size_t)g * gb;
        // edge records {nc, w, p, ev} (mz_tree_device.h)
        const uint32_t* rec = reinterpret_cast<const uint32_t*>(b);
        auto nc = [&](size_t i) { return rec[4 * i]; };
        auto w = [&](size_t i) { float v; std::memcpy(&v, rec + 4 * i + 1, 4); return v; };
        auto p = [&](size_t i) { float v; std::memcpy(&v, rec + 4 * i + 2, 4); return v; };
        const float* nr = reinterpret_cast<const float*>(b + 16 * (size_t)E);
        const int8_t* tp = reinterpret_cast<const int8_t*>(b + 16 * (size_t)E + 4 * (size_t)NN);
        // only expanded slots hold data: slot e is expanded iff e == 0 or some edge points at it
        std::vector<char> expd(NN, 0);
        expd[0] = 1;
        for (int i = 0; i < E; ++i) if ((nc(i) >> 16) != 0 && expd[i / A]) expd[(nc(i) >> 16) - 1] = 1;
        for (int e = 0; e < NN; ++e) {
            if (ntp) ntp[(size_t)g * NN + e] = expd[e] ? tp[e] : 0;
            for (int a = 0; a < A; ++a) {
                const size_t k = ((size_t)g * NN + e) * A + a, i = (size_t)e * A + a;
                const bool x = expd[e] != 0;
                const int c = x ? (int)(nc(i) >> 16) - 1 : -1;
                if (eN) eN[k] = x ? (int32_t)(nc(i) & 0xffffu) : 0;
                if (eW) eW[k] = x ? w(i) : 0.0f;
                if (eP) eP[k] = x ? p(i) : 0.0f;
                if (eR) eR[k] = c >= 0 ? nr[c] : 0.0f;
                if (eC) eC[k] = c;
            }
        }
    }
    return 0;
}

// ------------------------------------------------------------- learner
static int ensure_batch(mz_handle* h, int B) {
    if (B <= h->bcap) return 0;
    const int K = h->conf.num_unroll_steps, A = h->A;
    float** bufs[] = {&h->d_bobs, &h->d_bact, &h->d_btv, &h->d_btr, &h->d_btp, &h->d_bgs, &h->d_pv, &h->d_pp, &h->d_pr};
    size_t sizes[] = {(size_t)B * h->obs_feat, (size_t)B * (K + 1), (size_t)B * (K + 1), (size_t)B * (K + 1),
                      (size_t)B * (K + 1) * A, (size_t)B, (size_t)B * (K + 1), (size_t)B * (K + 1) * A,
                      (size_t)B * (K + 1)};
    for (int i = 0; i < 9; ++i) MZ_TRY(h, dalloc(h, bufs[i], sizes[i]));
    MZ_TRY(h, dalloc(h, &h->d_lterm, (size_t)2 * B * (K + 1)));
    MZ_TRY(h, dalloc(h, &h->d_bw, (size_t)B));
    if (h->kind == 1) {
        MZ_TRY(h, dalloc(h, &h->d_rhs, (size_t)B * std::max(K, 1) * h->H));
        MZ_TRY(h, dalloc(h, &h->d_rts, (size_t)B * std::max(K, 1) * h->H));
        MZ_TRY(h, dalloc(h, &h->d_prog, (size_t)B));
        MZ_TRY(h, hipMemset(h->d_prog, 0, (size_t)B * sizeof(unsigned long long)));
        h->prog_epoch = 0;
    }
    h->bcap = B;
    return 0;
}

static size_t runroll_lds(const mz_handle* h) {
    return std::max(h->rn_lds[0], std::max(h->rn_lds[1], h->rn_lds[2]));
}

static int learner_losses(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, hipStream_t st,
                          int v_act, int r_act, bool fuse_adam = false, double eta = 0.0, bool l2_done = false);
static void adam_advance(mz_handle* h);

// ResNet learner: the unroll on the network kernels, then the shared loss /
// ∇ = 2θ kernel (the plans' outputs are already activated)
static int rlearner_grad(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, void* stream,
                         bool fuse_adam = false, double eta = 0.0, const RpSampleParams* rq = nullptr) {
    const int B = b->batch_size;
    if (B < 1) return fail(h, "batch_size must be >= 1");
    if (ensure_batch(h, B)) return -1;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    RUnrollParams U;
    std::memset(&U, 0, sizeof(U));                 // (ms = 0: one step; the fused-ADAM fields unused unless set)
    U.B = B; U.K = h->conf.num_unroll_steps; U.A = h->A; U.H = h->H;
    U.W = h->rconf.observation_shape[0]; U.P = h->plane; U.obs_feat = h->rin_feat; U.ng = h->rn_ng; U.bn_s = h->bn_s;
    U.obs = b->observation; U.actions = b->actions;
    if (h->ds) {                                    // representation (:347): downsampler, then the tail
        if (ensure_dsb(h, B) || ds_launch(h, b->observation, h->d_dsb, B, st)) return -1;
        U.obs = h->d_dsb;
    } U.pv = h->d_pv; U.pp = h->d_pp; U.pr = h->d_pr;
    U.hs = h->d_rhs; U.plans = h->d_rplan; U.Wimg = h->d_Wp; U.flat = h->d_flat;
    U.plans_l = h->d_rplan_l; U.ng_l = h->rn_ng_l;
    U.dyn_split = h->rn_dyn_split; U.ts = h->d_rts; U.otab = h->d_rtab;
    U.stamps = nullptr;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, 128)));
    U.stamps = h->d_stamps;
#endif
    void* args[] = {&U};
    const int KH = std::max(U.K, 1);
    // the B·K predictions on wide tiles (ng items) once they fill the chip
    // (B = 2048: 640 workgroups; one-item tiles there measured 2.4x slower),
    // else one-item tiles (B = 32: 160 workgroups instead of 10)
    static const bool wide_env = std::getenv("MZ_RN_PRED_WIDE") != nullptr;
    static const bool one_kernel = std::getenv("MZ_RUNROLL_FUSED") != nullptr;
    const bool wide_p = wide_env || (B * KH + U.ng - 1) / U.ng >= h->n_cu;
    // one launch (mz_runroll_fused_r): the chain blocks, then the items, each
    // item waiting for its sample's chain instead of the whole launch; with
    // rq, each chain block also draws its sample (the get_batch launch folded in)
    static const bool no_fuse = std::getenv("MZ_RN_NO_FUSE") != nullptr;
    const bool fused = !one_kernel && h->rd_chain && h->rp_pred && !wide_p && !no_fuse && U.ng_l == 1 &&
                       U.K + 1 < 64 && !h->ds && h->d_prog;
    static const bool no_fuse_sample = std::getenv("MZ_RN_NO_FUSE_SAMPLE") != nullptr;   // A/B only
    static const bool no_fuse_adam = std::getenv("MZ_RN_NO_FUSE_ADAM") != nullptr;       // A/B only
    bool l2_fused = false;
    if (rq && (!fused || no_fuse_sample)) {
        hipLaunchKernelGGL(mz_rp_sample, dim3((B + 3) / 4), dim3(256), 0, st, *rq);
        MZ_TRY(h, hipGetLastError());
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->time_unroll) {
        if (timing_events(h, &e0, &e1)) return -1;
        MZ_TRY(h, hipEventRecord(e0, st));
    }
    if (one_kernel) {          // the one-kernel unroll (pred inside the chain)
        h->last_lvariant = "mz_runroll_kernel";
        MZ_TRY(h, hipLaunchKernel((const void*)mz_runroll_kernel, dim3((B + U.ng - 1) / U.ng), dim3(RN_THREADS),
                                  args, runroll_lds(h), st));
    } else {                                        // chain on narrow tiles, then the B·K predictions
        // units of one column block (the 1-block instances, a fifth of the code),
        // also for wider tiles: a Connect4 1x1 conv of 4 row blocks x 3 column
        // blocks then has 12 units for the 8 waves instead of 4 three-block ones
        // (the same tiles, bit for bit; configs[3] learner 1.62 k -> 1.75 k
        // steps/s, tools/gpu_r04d.sh).  MZ_RN_CHAIN_NB3=1: the three-block units
        static const bool nb3 = std::getenv("MZ_RN_CHAIN_NB3") != nullptr;
        const bool nb1 = (U.P * U.ng_l + 15) / 16 == 1 || !nb3;
        U.rd_ep_off = (int)(h->rn_lds_l / 4);
        U.rd_trunk_nl = 1 + 2 * h->rhp.num_blocks;
        h->last_lvariant = std::string(h->rd_chain ? (h->rd_nb == 3 ? "mz_runroll_chain_r3" : "mz_runroll_chain_r")
                                                   : nb1 ? "mz_runroll_chain1" : "mz_runroll_chain") +
                           (wide_p ? "+mz_runroll_pred" : h->rp_pred ? "+mz_runroll_pred_r" : nb1 ? "+mz_runroll_pred_n1"
                                                                                       : "+mz_runroll_pred_n");
        if (fused) {
            U.prog = h->d_prog;
            U.prog_base = (++h->prog_epoch) * 64ull;
            U.fault = h->d_fault; U.poll_ticks = h->poll_ticks; U.dbg_skip = h->dbg_skip;
            U.n_chain = B;
            U.fuse_sample = rq != nullptr && !no_fuse_sample;
            if (rq) U.rq = *rq;
            // ADAM beside the unroll: the launch reads the current image (d_Wp) and
            // writes the updated one into d_Wp2, swapped after the launch
            U.n_l2 = fuse_adam && h->d_Wp2 && !no_fuse_adam ? 96 : 0;
            U.ad = LgAdam{1, h->d_m, h->d_v, h->bp1, h->bp2, eta, h->d_Wp2, h->d_Bp, h->d_inv_tile, nullptr,
                          nullptr, h->d_inv_small};
            U.flat_w = h->d_flat; U.netoff = h->d_netoff; U.part = h->d_sq;
            l2_fused = U.n_l2 > 0;
            h->last_lvariant = h->rd_nb == 3 ? "mz_runroll_fused_r3" : "mz_runroll_fused_r";
            U.rp_nv = 3 + h->rhp.depth_value;       // value head: conv, Dense, depth_value × Dense, Dense
            const int nitems = B * KH * (U.K > 0 ? 3 : 2);
            MZ_TRY(h, hipLaunchKernel(h->rd_nb == 3 ? (const void*)mz_runroll_fused_r3 : (const void*)mz_runroll_fused_r,
                                      dim3(B + U.n_l2 + nitems), dim3(RD_THREADS), args,
                                      std::max(rd_chain_lds(h), rp_pred_lds(h)), st));
        } else if (h->rd_chain)
            MZ_TRY(h, hipLaunchKernel(h->rd_nb == 3 ? (const void*)mz_runroll_chain_r3 : (const void*)mz_runroll_chain_r,
                                      dim3((B + U.ng_l - 1) / U.ng_l),
                                      dim3(RD_THREADS), args, rd_chain_lds(h), st));
        else
            MZ_TRY(h, hipLaunchKernel(nb1 ? (const void*)mz_runroll_chain1 : (const void*)mz_runroll_chain,
                                      dim3((B + U.ng_l - 1) / U.ng_l), dim3(RN_THREADS),
                                      args, h->rn_lds_l, st));
        // the B·K predictions and reward heads (wide_p above)
        if (fused) {
        } else if (wide_p)
            MZ_TRY(h, hipLaunchKernel((const void*)mz_runroll_pred, dim3((B * KH + U.ng - 1) / U.ng, U.K > 0 ? 2 : 1),
                                      dim3(RN_THREADS), args, runroll_lds(h), st));
        else if (h->rp_pred)
            MZ_TRY(h, hipLaunchKernel((const void*)mz_runroll_pred_r, dim3((B * KH + U.ng_l - 1) / U.ng_l,
                                      U.K > 0 ? 2 : 1), dim3(RD_THREADS), args, rp_pred_lds(h), st));
        else
            MZ_TRY(h, hipLaunchKernel(nb1 ? (const void*)mz_runroll_pred_n1 : (const void*)mz_runroll_pred_n,
                                      dim3((B * KH + U.ng_l - 1) / U.ng_l, U.K > 0 ? 2 : 1), dim3(RN_THREADS), args,
                                      h->rn_lds_l, st));
    }
    if (e1) MZ_TRY(h, hipEventRecord(e1, st));
    if (learner_losses(h, b, grad_dev, losses_dev, st, MZ_ACT_IDENTITY, MZ_ACT_IDENTITY, fuse_adam, eta, l2_fused))
        return -1;
    if (l2_fused) {
        std::swap(h->d_Wp, h->d_Wp2);
        adam_advance(h);
    }
    return 0;
}

static int fc_unroll(mz_handle* h, const mz_batch* b, hipStream_t st, const RpSampleParams* rp);
static int bp_grad(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, hipStream_t st);
static int small_unroll_ti(const mz_handle* h, int B);
static int small_unroll_params(mz_handle* h, const mz_batch* b, int ti, const RpSampleParams* rp,
                               SmallUnrollParams* Uo);

// forward unroll + losses + ∇ = 2θ into grad_dev (device batch pointers)
int mz_learner_grad_dev(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, void* stream) {
    if (!h || !b) return -2;
    if (b->batch_size < 1) return fail(h, "batch_size must be >= 1");
    if (h->learn_mode == MZ_LEARN_CORRECTED)
        return bp_grad(h, b, grad_dev, losses_dev, stream ? (hipStream_t)stream : h->stream);
    if (h->kind == 1) return rlearner_grad(h, b, grad_dev, losses_dev, stream);
    if (ensure_batch(h, b->batch_size)) return -1;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if (fc_unroll(h, b, st, nullptr)) return -1;
    return learner_losses(h, b, grad_dev, losses_dev, st, h->lay.v_act, h->lay.r_act);
}

// FC learner unroll of batch b (Learning.jl:327-343); rp != nullptr: the
// batch is drawn from the replay shard by get_batch (mz_rp_sample's body),
// inside the small unroll kernel when it applies, else by its own launch
static int fc_unroll(mz_handle* h, const mz_batch* b, hipStream_t st, const RpSampleParams* rp) {
    const int B = b->batch_size, K = h->conf.num_unroll_steps, A = h->A;
    const int ti_u = small_unroll_ti(h, B);
    if (ti_u >= 0) {
        // the search's stage schedule and register images, T samples per
        // workgroup (ADAM keeps the images current)
        const int ti = ti_u, T = ti + 1;
        SmallUnrollParams U;
        if (small_unroll_params(h, b, ti, rp, &U)) return -1;
        void* args[] = {&U};
        MZ_TRY(h, hipLaunchKernel(h->sm_bn ? (ti == 0 ? (const void*)mz_unroll_small1_bn : (const void*)mz_unroll_small2_bn)
                                           : (ti == 0 ? (const void*)mz_unroll_small1 : (const void*)mz_unroll_small2),
                                  dim3((B + T - 1) / T), dim3(SM_THREADS), args, unroll_small_lds(h, ti), st));
        h->last_lvariant = ti == 0 ? "mz_unroll_small1" : "mz_unroll_small2";
    } else {
        if (rp) {
            hipLaunchKernelGGL(mz_rp_sample, dim3((B + 3) / 4), dim3(256), 0, st, *rp);
            MZ_TRY(h, hipGetLastError());
        }
        UnrollParams U;
        U.B = B; U.K = K; U.A = A; U.H = h->H; U.plane = h->plane; U.obs_feat = h->obs_feat;
        U.obs = b->observation; U.actions = b->actions; U.pv = h->d_pv; U.pp = h->d_pp; U.pr = h->d_pr;
        U.Wp = h->d_Wp; U.Bp = h->d_Bp; U.plan_repr = h->d_plan[0]; U.plan_sim = h->d_plan[4]; U.lay = h->lay;
        hipLaunchKernelGGL(mz_unroll_kernel, dim3((B + MZ_TILE - 1) / MZ_TILE), dim3(MZ_THREADS),
                           (size_t)h->lay.total * 4, st, U);
        h->last_lvariant = "mz_unroll_kernel";
    }
    MZ_TRY(h, hipGetLastError());
    return 0;
}

// the small unroll holds the nets with T = ti + 1 samples per workgroup
static bool small_unroll_fits(const mz_handle* h, int ti) {
    const int K = h->conf.num_unroll_steps, A = h->A;
    // one item per thread in the unroll's per-step loops; a/|A| staging of 64 floats
    return h->small_ok && (ti + 1) * h->H <= 256 && (ti + 1) * h->plane <= 256 &&
           (ti + 1) * (A + 2) <= SM_THREADS && (ti + 1) * (K + 1) <= 64 &&
           (ti + 1) * h->obs_feat <= SM_THREADS;                // one observation item per thread (setup)
}
// T = 2 when B exceeds 4 samples per CU; -1 if the small unroll cannot hold the nets
static int small_unroll_ti(const mz_handle* h, int B) {
    const int ti_u = B <= 4 * h->n_cu ? 0 : 1;         // (two per workgroup at B = 32: 29.5 k vs 34.0 k steps/s)
    return small_unroll_fits(h, ti_u) ? ti_u : -1;
}

// parameters of mz_unroll_small* / mz_learn_small* for batch b (T = ti + 1
// samples per workgroup, the search's stage schedule and register images)
static int small_unroll_params(mz_handle* h, const mz_batch* b, int ti, const RpSampleParams* rp,
                               SmallUnrollParams* Uo) {
    const int B = b->batch_size, K = h->conf.num_unroll_steps, A = h->A;
    {
        const int* lay = h->sm_lay[ti];
        SmallUnrollParams U;
        U.B = B; U.K = K; U.A = A; U.H = h->H; U.plane = h->plane; U.obs_feat = h->obs_feat;
        U.obs = b->observation; U.actions = b->actions; U.pv = h->d_pv; U.pp = h->d_pp; U.pr = h->d_pr;
        U.n_sim = h->sm_n_sim; U.n_root = h->sm_n_root; U.w_sim = h->d_sm_w;
        U.w_root = h->d_sm_w + (size_t)h->sm_n_sim * SM_SLOTS * 256 * 16;
        std::memcpy(U.nzm, h->sm_nzm.data(), sizeof(U.nzm));
        U.bn = h->sm_bn;
        U.zero16 = reinterpret_cast<const float4*>(h->d_zero16);
        U.bias = h->d_sm_bias; U.rec = h->d_sm_rec[ti]; U.act_total = lay[0];
        U.x_rep = lay[1]; U.x_pred = lay[2]; U.x_dyn = lay[3]; U.h_out = lay[4]; U.v_out = lay[5];
        U.p_out = lay[6]; U.r_out = lay[7]; U.v_act = h->lay.v_act; U.r_act = h->lay.r_act;
        U.stamps = nullptr;
#ifdef MZ_STAMPS
        if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, B)));
        U.stamps = h->d_stamps;
#endif
        U.sample = rp != nullptr;
        U.pf_hdr = nullptr; U.pf_epoch = 0;
        if (rp) U.rp = *rp; else std::memset(&U.rp, 0, sizeof(U.rp));
        *Uo = U;
    }
    return 0;
}

static LgAdam adam_args(mz_handle* h, int on, double eta) {
    return LgAdam{on, h->d_m, h->d_v, h->bp1, h->bp2, eta, h->d_Wp, h->d_Bp, h->d_inv_tile, h->d_sm_w,
                  h->d_sm_bias, h->d_inv_small};
}
// after an ADAM update: βp .= βp .* β
static void adam_advance(mz_handle* h) {
    h->bp1 = h->bp1 * 0.9;
    h->bp2 = h->bp2 * 0.999;
}

// losses + ∇ = 2θ from the unroll outputs in d_pv / d_pp / d_pr; with
// fuse_adam (world = 1) the ∇ is not stored: each parameter slice's block
// applies the ADAM update (learning rate eta) right after reading θ for Σθ²
static int learner_losses(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, hipStream_t st,
                          int v_act, int r_act, bool fuse_adam, double eta, bool l2_done) {
    const int B = b->batch_size, K = h->conf.num_unroll_steps, A = h->A;
    float* lo = losses_dev ? losses_dev : h->d_loss;
    float* g = grad_dev ? grad_dev : h->d_grad;
    const int gw = A > 16 ? 32 : 16;            // lanes per (sample, step) group
    const int nlb = (B * (K + 1) + MZ_THREADS / gw - 1) / (MZ_THREADS / gw);
    const LgAdam ad = adam_args(h, fuse_adam ? 1 : 0, eta);
    // l2_done: the Σθ² slices (and the ADAM step) ran in the unroll launch; only the loss blocks and the fold
    hipLaunchKernelGGL(gw == 32 ? mz_learner_grad_kernel32 : mz_learner_grad_kernel,
                       dim3(nlb + (l2_done ? 0 : 3 * MZ_L2_BLOCKS)), dim3(MZ_THREADS), 0, st, B, K, A,
                       v_act, r_act, h->d_pv, h->d_pp, h->d_pr, b->target_values, b->target_policies,
                       b->gradient_scale, h->d_lterm, h->d_flat, h->d_netoff, g, h->d_sq, h->d_counter, lo, b->weights, ad);
    MZ_TRY(h, hipGetLastError());
    if (fuse_adam && !l2_done) adam_advance(h);
    return 0;
}

// ---- corrected-gradient learner (MZ_LEARN_CORRECTED, FC nets; mz_backprop.hip)
// The unrolled graph of Learning.jl:347-370: representation(obs); K dynamics
// steps on sa_k = [2h_{k-1} ; a_{k-1}/|A|] (the state head skipped at k = K,
// whose h_K no prediction reads; the reward heads only with
// intermediate_rewards); K+1 predictions on h_0, h_0, h_1 .. h_{K-1} (Q10).
static int build_bp(mz_handle* h) {
    const int K = h->conf.num_unroll_steps, H = h->H;
    std::vector<BpApp> apps;
    std::vector<BpHead> heads;
    int off = 0;
    auto tensor = [&](int rows) { int o = off; off += ((rows + 3) & ~3) * 16; return o; };
    const int obs_t = tensor(h->obs_feat);
    auto dense = [&](int li, int x) {
        const LayerSpec& L = h->layers[li];
        BpApp a{};
        a.op = BP_DENSE; a.w_off = (int)L.flux_w; a.b_off = (int)L.flux_b; a.in = L.in; a.out = L.out;
        a.act = L.act; a.x = x; a.y = tensor(L.out); a.step = li;
        a.bn_off = L.bn ? (int)L.flux_be : -1;                // make_dense's BatchNorm: t kept at z
        a.z = L.bn ? tensor(L.out) : -1;
        apps.push_back(a);
        return a.y;
    };
    auto chain = [&](int net, int ch, int x) {
        for (int li : h->chains[net][ch]) x = dense(li, x);
        return x;
    };
    std::vector<int> hs(K + 1, -1);
    hs[0] = chain(MZ_NET_REPR, CH_TRUNK, obs_t);                                // :347
    for (int k = 1; k <= K; ++k) {                                              // :355-362
        BpApp c{};
        c.op = BP_CONCAT; c.in = H; c.out = H + h->plane; c.x = hs[k - 1]; c.y = tensor(c.out); c.step = k - 1;
        c.bn_off = c.z = -1;
        apps.push_back(c);
        const int t = chain(MZ_NET_DYN, CH_TRUNK, c.y);
        if (k < K) hs[k] = chain(MZ_NET_DYN, CH_HEAD1, t);
        if (h->conf.intermediate_rewards) heads.push_back(BpHead{BP_HEAD_R, chain(MZ_NET_DYN, CH_HEAD2, t), k});
    }
    for (int k = 0; k <= K; ++k) {                                              // :351, :356 (Q10)
        const int t = chain(MZ_NET_PRED, CH_TRUNK, hs[k <= 1 ? 0 : k - 1]);
        heads.push_back(BpHead{BP_HEAD_V, chain(MZ_NET_PRED, CH_HEAD1, t), k});
        heads.push_back(BpHead{BP_HEAD_P, chain(MZ_NET_PRED, CH_HEAD2, t), k});
    }
    // level schedule of the tile kernel (mz_bp_tile_lv).  Forward: an
    // application's level is one past its input's producer (the observation:
    // level 0).  Backward, in reverse application order: one past the latest
    // consumer of its output (the applications reading it, which accumulate
    // G[y]), and past every later application accumulating into the same G[x]
    // (so no two units of a level add into one tensor, and the sequential
    // kernel's accumulation order holds)
    const int na = (int)apps.size();
    std::vector<int> flv(na, 0), blv(na, 0);
    int nfl = 0, nbl = 0;
    for (int a = 0; a < na; ++a) {
        int l = 0;
        for (int p = 0; p < a; ++p) if (apps[p].y == apps[a].x) l = std::max(l, flv[p] + 1);
        flv[a] = l; nfl = std::max(nfl, l + 1);
    }
    for (int a = na - 1; a >= 0; --a) {
        int l = 0;
        for (int c = a + 1; c < na; ++c) {
            if (apps[c].x == apps[a].y) l = std::max(l, blv[c] + 1);           // consumers of y
            if (apps[c].x == apps[a].x) l = std::max(l, blv[c] + 1);           // same G[x], earlier in backward
        }
        blv[a] = l; nbl = std::max(nbl, l + 1);
    }
    // ... then each backward application as late as those constraints allow
    // (the same level count): ASAP piles every prediction head of the unroll
    // into the first levels (~70 units on 16 waves, serialised), ahead of the
    // dynamics chain they do not gate; ALAP spreads them along the chain.
    // Application c must precede a (a < c) when a produces c's input or adds
    // into the same G[x] after it.  MZ_BP_ASAP=1 keeps the ASAP levels.
    if (!std::getenv("MZ_BP_ASAP")) {
        for (int c = 0; c < na; ++c) {
            int l = nbl - 1;
            for (int a = 0; a < c; ++a)
                if (apps[c].x == apps[a].y || apps[c].x == apps[a].x) l = std::min(l, blv[a] - 1);
            blv[c] = l;
        }
    }
    std::vector<int2> fun, bun;
    std::vector<int> flev, blev;
    for (int l = 0; l < nfl; ++l) {
        flev.push_back((int)fun.size());
        for (int a = 0; a < na; ++a)
            if (flv[a] == l) {
                const int nb = apps[a].op == BP_DENSE ? (apps[a].out + 15) / 16 : 1;
                for (int b = 0; b < nb; ++b) fun.push_back(make_int2(a, b));
            }
    }
    flev.push_back((int)fun.size());
    for (int l = 0; l < nbl; ++l) {
        blev.push_back((int)bun.size());
        for (int a = na - 1; a >= 0; --a)
            if (blv[a] == l) {
                const int nb = apps[a].op == BP_DENSE ? (apps[a].in + 15) / 16 : 1;
                for (int b = 0; b < nb; ++b) bun.push_back(make_int2(a, b));
            }
    }
    blev.push_back((int)bun.size());
    // mz_bp_tile_lv's LDS tensor cache: slots of the largest tensor.  Forward,
    // level by level: a tensor read at later levels takes a free slot when it
    // is produced (its readers read the copy) and frees it after its last
    // reading level.  Backward: a ∂L/∂x takes a slot at its first contribution
    // and frees it after its producer's level read it (and wrote it out for
    // mz_bp_dw).  Everything else stays in the arena: the level that writes it
    // ends with a barrier that drains the stores (fsync / bsync), as do the
    // last forward level (the heads and the backward read the arena).
    std::vector<int> fsync(nfl, 0), bsync(nbl, 0);
    int cache_floats = 0, obs_s = -1;
    for (BpApp& a : apps) { a.xs = a.ys = a.gys = a.gxs = -1; a.gxf = 0; }
#if BP_LV_SIMPLE && !BP_LV_PREFETCH
    {
        auto rows16 = [](int r) { return ((r + 3) & ~3) * 16; };
        int slot = rows16(h->obs_feat);
        for (const BpApp& a : apps) slot = std::max(slot, rows16(a.out));
        const size_t sched = (size_t)na * sizeof(BpApp) + (fun.size() + bun.size()) * sizeof(int2) +
                             (size_t)(2 * (nfl + nbl) + 8) * sizeof(int);
        // (a schedule that leaves no room for the cache runs without it, not with a wrapped count)
        const int nslot = sched + 64 < kLdsMax
                              ? (int)std::min<size_t>(64, (kLdsMax - sched - 64) / ((size_t)slot * 4)) : 0;
        cache_floats = nslot * slot;
        std::vector<int> free_s;
        for (int i = nslot - 1; i >= 0; --i) free_s.push_back(i * slot);
        // forward
        std::map<int, int> last_read, fslot;                 // tensor -> last reading level, -> slot
        for (int a = 0; a < na; ++a) last_read[apps[a].x] = std::max(last_read.count(apps[a].x) ? last_read[apps[a].x] : -1, flv[a]);
        auto take = [&](int t) {
            if (!last_read.count(t) || free_s.empty()) return -1;
            const int o = free_s.back(); free_s.pop_back();
            fslot[t] = o;
            return o;
        };
        obs_s = take(obs_t);
        for (int l = 0; l < nfl; ++l) {
            for (auto it = fslot.begin(); it != fslot.end();) {
                if (last_read[it->first] < l) { free_s.push_back(it->second); it = fslot.erase(it); }
                else ++it;
            }
            for (int a = 0; a < na; ++a)
                if (flv[a] == l) { auto f = fslot.find(apps[a].x); apps[a].xs = f != fslot.end() ? f->second : -1; }
            for (int a = 0; a < na; ++a)
                if (flv[a] == l) {
                    apps[a].ys = take(apps[a].y);
                    if (apps[a].ys < 0 && last_read.count(apps[a].y)) fsync[l] = 1;
                }
        }
        fsync[nfl - 1] = 1;
        // backward
        free_s.clear();
        for (int i = nslot - 1; i >= 0; --i) free_s.push_back(i * slot);
        std::map<int, int> producer, where, gslot;            // tensor -> app, -> slot or -1 (decided), live slots
        for (int a = 0; a < na; ++a) producer[apps[a].y] = a;
        for (const BpHead& hd : heads) where[hd.y] = -1;      // bp_heads writes these to the arena
        for (int l = 0; l < nbl; ++l) {
            for (auto it = gslot.begin(); it != gslot.end();) {
                if (blv[producer[it->first]] < l) { free_s.push_back(it->second); it = gslot.erase(it); }
                else ++it;
            }
            for (int a = 0; a < na; ++a) {
                if (blv[a] != l) continue;
                auto g = gslot.find(apps[a].y);
                apps[a].gys = g != gslot.end() ? g->second : -1;
            }
            for (int a = 0; a < na; ++a) {
                if (blv[a] != l) continue;
                const int t = apps[a].x;
                auto w = where.find(t);
                if (w == where.end()) {
                    int o = -1;
                    if (producer.count(t) && !free_s.empty()) {
                        o = free_s.back(); free_s.pop_back();
                        gslot[t] = o;
                        apps[a].gxf = 1;
                    }
                    where[t] = o;
                    apps[a].gxs = o;
                } else {
                    apps[a].gxs = w->second;
                }
                if (apps[a].gxs < 0) bsync[l] = 1;
            }
        }
    }
#endif
    // dW: every layer's applications, one wave per 16x16 block (+ one per bias block)
    std::vector<BpLayer> layers(h->layers.size());
    std::vector<BpUse> uses;
    std::vector<BpJob> jobs;
    for (int n = 0; n < 4; ++n) h->bp_job0[n] = -1;
    for (size_t li = 0; li < h->layers.size(); ++li) {
        const LayerSpec& L = h->layers[li];
        if (h->bp_job0[L.net] < 0) h->bp_job0[L.net] = (int)jobs.size();   // layers are in net order
        BpLayer& bl = layers[li];
        bl.w_off = (int)L.flux_w; bl.b_off = (int)L.flux_b; bl.in = L.in; bl.out = L.out; bl.act = L.act;
        bl.bn_off = L.bn ? (int)L.flux_be : -1;
        bl.use0 = (int)uses.size();
        for (const BpApp& a : apps) if (a.op == BP_DENSE && a.step == (int)li) uses.push_back(BpUse{a.x, a.y, a.z});
        bl.n_use = (int)uses.size() - bl.use0;
        for (int ob = 0; ob < (L.out + 15) / 16; ++ob) {
            for (int ib = 0; ib < (L.in + 15) / 16; ++ib) jobs.push_back(BpJob{(int)li, ob, ib});
            jobs.push_back(BpJob{(int)li, ob, -1});
        }
    }
    auto up = [&](auto** d, const auto& v) -> int {
        MZ_TRY(h, dalloc(h, d, v.size()));
        MZ_TRY(h, hipMemcpy(*d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice));
        return 0;
    };
    if (up(&h->d_bp_apps, apps) || up(&h->d_bp_heads, heads) || up(&h->d_bp_layers, layers) ||
        up(&h->d_bp_uses, uses) || up(&h->d_bp_jobs, jobs) || up(&h->d_bp_funits, fun) ||
        up(&h->d_bp_flev, flev) || up(&h->d_bp_bunits, bun) || up(&h->d_bp_blev, blev) ||
        up(&h->d_bp_fsync, fsync) || up(&h->d_bp_bsync, bsync))
        return -1;
    h->bp_cache_floats = cache_floats; h->bp_obs_s = obs_s;
    {
        const size_t lv = (size_t)na * sizeof(BpApp) + (fun.size() + bun.size()) * sizeof(int2) +
                          (size_t)(2 * (nfl + nbl) + 8) * sizeof(int) + 16 + (size_t)cache_floats * 4;
        if (lv > kLdsMax) return fail(h, "corrected learner: the level schedule exceeds the LDS");
        MZ_TRY(h, hipFuncSetAttribute((const void*)mz_bp_tile_lv, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lv));
        MZ_TRY(h, hipFuncSetAttribute((const void*)mz_bp_tile_lv_nobn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lv));
    }
    h->bp_n_flev = nfl; h->bp_n_blev = nbl; h->bp_n_funit = (int)fun.size(); h->bp_n_bunit = (int)bun.size();
    h->bp_n_app = (int)apps.size(); h->bp_n_head = (int)heads.size(); h->bp_n_job = (int)jobs.size();
    h->bp_job0[3] = (int)jobs.size();
    for (int n = 2; n >= 0; --n) if (h->bp_job0[n] < 0) h->bp_job0[n] = h->bp_job0[n + 1];
    MZ_TRY(h, dalloc(h, &h->d_bp_sq, jobs.size()));
    h->bp_tile_floats = off; h->bp_obs_t = obs_t;
    h->bp_built = true;
    return 0;
}

// ---- the corrected learner for the ResNet nets (mz_backprop.hip mz_rbp_*):
// the same unrolled graph as build_bp, on the layers of rn_specs (convs with
// BatchNorm and residual blocks, the heads' 1x1 convs, Dense layers), one
// arena per sample: conv tensors [channel][position], dense vectors.
static int build_rbp(mz_handle* h) {
    const int K = h->conf.num_unroll_steps, P = h->plane, H = h->H;
    std::vector<RbpApp> apps;
    std::vector<BpHead> heads;
    int off = 0, dtf = 0, xsf = 0, max_units = 1;
    auto tensor = [&](int n) { int o = off; off += (n + 3) & ~3; return o; };
    const int obs_t = tensor(h->rin_feat);
    std::vector<RSpec> sp[3];
    size_t np[3];
    for (int n = 0; n < 3; ++n) sp[n] = rn_specs(h->rconf, h->rhp, n, &np[n]);
    // one RbpLayer per spec (nets in order) and its applications
    int lbase[3], nl = 0;
    for (int n = 0; n < 3; ++n) { lbase[n] = nl; nl += (int)sp[n].size(); }
    std::vector<std::vector<RbpUse>> luse(nl);
    const int npb = (P + 15) / 16;
    // the representation's tail follows the downsampler's parameters in net 0
    auto fo = [&](int net) { return h->flat_off[net] + (net == MZ_NET_REPR && h->ds ? h->ds_n : 0); };
    auto chain = [&](int net, int ch, int x, bool first_obs) {
        int saved = -1;
        for (size_t si = 0; si < sp[net].size(); ++si) {
            const RSpec& r = sp[net][si];
            if (r.chain != ch) continue;
            RbpApp a{};
            a.op = r.conv ? RBP_CONV : RBP_DENSE;
            a.w_off = (int)(fo(net) + r.woff); a.b_off = (int)(fo(net) + r.boff);
            a.bn_off = r.conv && r.bn ? (int)(fo(net) + r.bnoff) : -1;
            a.cin = r.cin; a.cout = r.cout; a.kw = r.kw; a.kh = r.kh; a.act = r.act;
            a.x = x; a.y = tensor(r.conv ? r.cout * P : r.cout);
            a.z = a.bn_off >= 0 ? tensor(r.cout * P) : -1;
            a.res = r.res_add ? saved : -1;
            if (r.res_save) saved = x;
            a.step = first_obs ? 1 : 0;
            first_obs = false;
            dtf = std::max(dtf, r.conv ? r.cout * P : r.cout);
            xsf = std::max(xsf, r.conv ? r.cin * P : r.cin);             // the staged input
            if (r.conv && r.kw * r.kh > 1) {                                // padded (mz_backprop.hip rbp_taps)
                const int Wb = h->rconf.observation_shape[0], Pp = (P / Wb + r.kh - 1) * (Wb + r.kw - 1);
                xsf = std::max(xsf, r.cin * Pp);
                dtf = std::max(dtf, r.cout * Pp);
            }
            if (r.conv) {
                max_units = std::max(max_units, std::max((r.cout + 15) / 16, (r.cin + 15) / 16) * npb);
            }
            apps.push_back(a);
            luse[lbase[net] + (int)si].push_back(RbpUse{a.x, a.y, a.z});
            x = a.y;
        }
        return x;
    };
    std::vector<int> hs(K + 1, -1);
    // :347; with the downsampler the first conv also produces ∂L/∂(its input) for mz_dsbp_bwd
    hs[0] = chain(MZ_NET_REPR, 0, obs_t, !h->ds);
    for (int k = 1; k <= K; ++k) {                                              // :355-362
        RbpApp c{};
        c.op = RBP_CONCAT; c.cin = H; c.cout = H + P; c.x = hs[k - 1]; c.y = tensor(c.cout); c.step = k - 1;
        c.bn_off = -1; c.z = -1; c.res = -1;
        dtf = std::max(dtf, c.cout);                                            // a ring slot holds it too
        apps.push_back(c);
        const int t = chain(MZ_NET_DYN, 0, c.y, false);
        if (k < K) hs[k] = chain(MZ_NET_DYN, 1, t, false);
        if (h->conf.intermediate_rewards) heads.push_back(BpHead{BP_HEAD_R, chain(MZ_NET_DYN, 2, t, false), k});
    }
    for (int k = 0; k <= K; ++k) {                                              // :351, :356 (Q10)
        const int t = chain(MZ_NET_PRED, 0, hs[k <= 1 ? 0 : k - 1], false);
        heads.push_back(BpHead{BP_HEAD_V, chain(MZ_NET_PRED, 1, t, false), k});
        heads.push_back(BpHead{BP_HEAD_P, chain(MZ_NET_PRED, 2, t, false), k});
    }
    // mz_rbp_sample's forward LDS ring: application a's output also goes to slot
    // a mod ns; an input or residual produced fewer than ns applications earlier
    // is read there, anything else from the arena, after a barrier that drained
    // the arena stores (fsync on the application before; the backward and the
    // heads read the arena too)
    const int ysz = (dtf + 3) & ~3, xsz = (xsf + 3) & ~3;
    int ns = 4;
    while (ns > 0 && (size_t)(ysz + xsz + ns * ysz) * 4 > kLdsMax) --ns;
    {
        std::map<int, int> producer;
        for (int a = 0; a < (int)apps.size(); ++a) {
            RbpApp& A_ = apps[a];
            auto slot = [&](int t) {
                auto it = producer.find(t);
                return it != producer.end() && a - it->second < ns ? it->second % ns : -1;
            };
            A_.xb = slot(A_.x);
            A_.rb = A_.res >= 0 ? slot(A_.res) : -1;
            A_.yb = ns > 0 ? a % ns : -1;
            A_.fsync = 0;
            if ((A_.xb < 0 || (A_.res >= 0 && A_.rb < 0)) && a > 0) apps[a - 1].fsync = 1;
            producer[A_.y] = a;
        }
        apps.back().fsync = 1;
    }
    // the backward ring (the same slots): in backward order, a tensor's ∂L/∂·
    // takes a free slot at its first contribution when its producer follows
    // within kGLife applications, and frees it when the producer has read it;
    // otherwise it accumulates in the arena (zeroed first, bsync after each
    // contribution).  The accumulation order is the arena's.
    std::vector<int2> gz;
    {
        const int kGLife = 6;
        std::map<int, int> producer, size_of;
        for (int a = 0; a < (int)apps.size(); ++a) {
            producer[apps[a].y] = a;
            size_of[apps[a].y] = apps[a].op == RBP_CONV ? apps[a].cout * P : apps[a].cout;
        }
        std::map<int, int> slot_of;          // tensor -> slot (ring-resident, live)
        std::map<int, int> where;            // tensor -> slot or -1 (decided at the first contribution)
        std::vector<int> free_slots;
        for (int i = ns - 1; i >= 0; --i) free_slots.push_back(i);
        for (int a = (int)apps.size() - 1; a >= 0; --a) {
            RbpApp& A_ = apps[a];
            A_.gyb = A_.gxb = A_.grb = -1; A_.gxf = A_.grf = 0; A_.bsync = 0;
            auto it = slot_of.find(A_.y);
            if (it != slot_of.end()) A_.gyb = it->second;
            auto contribute = [&](int t, int& sb, int& first) {
                auto w = where.find(t);
                if (w == where.end()) {
                    auto pr = producer.find(t);
                    int sl = -1;
                    if (pr != producer.end() && a - pr->second <= kGLife && !free_slots.empty()) {
                        sl = free_slots.back(); free_slots.pop_back();
                        slot_of[t] = sl;
                        first = 1;
                    }
                    where[t] = sl;
                    sb = sl;
                } else {
                    sb = w->second;
                }
                if (sb < 0) A_.bsync = 1;
            };
            const bool dx = A_.op == RBP_CONCAT || !A_.step;
            if (dx) contribute(A_.x, A_.gxb, A_.gxf);
            if (A_.op == RBP_CONV && A_.res >= 0) contribute(A_.res, A_.grb, A_.grf);
            if (A_.gyb >= 0) { free_slots.push_back(A_.gyb); slot_of.erase(A_.y); }
        }
        for (const auto& t : size_of)
            if (where.find(t.first) == where.end() || where[t.first] < 0) gz.push_back(make_int2(t.first, t.second));
        if (h->ds) gz.push_back(make_int2(obs_t, h->rin_feat));
    }
    h->rbp_ring = ns;
    // mz_rbp_dw's jobs, net by net (mz_bp_fold sums each net's Σθ² over its job range):
    // per layer its W blocks, then its bias (BatchNorm) blocks; every parameter once
    std::vector<RbpLayer> layers(nl);
    std::vector<RbpUse> uses;
    std::vector<RbpJob> jobs;
    std::vector<char> covered(h->nflat, 0);
    for (int n = 0; n < 3; ++n) {
        h->rbp_job0[n] = (int)jobs.size();
        for (size_t si = 0; si < sp[n].size(); ++si) {
            const RSpec& r = sp[n][si];
            const int li = lbase[n] + (int)si;
            RbpLayer& L = layers[li];
            L.conv = r.conv; L.w_off = (int)(fo(n) + r.woff); L.b_off = (int)(fo(n) + r.boff);
            L.bn_off = r.conv && r.bn ? (int)(fo(n) + r.bnoff) : -1;
            L.cin = r.cin; L.cout = r.cout; L.kw = r.kw; L.kh = r.kh; L.act = r.act;
            L.use0 = (int)uses.size(); L.n_use = (int)luse[li].size();
            for (const RbpUse& u : luse[li]) uses.push_back(u);
            const int Kw = r.conv ? r.kw * r.kh * r.cin : r.cin;
            for (int ob = 0; ob < (r.cout + 15) / 16; ++ob)
                for (int kb = 0; kb < (Kw + 15) / 16; ++kb) jobs.push_back(RbpJob{li, ob, kb});
            for (int ob = 0; ob < (r.cout + 15) / 16; ++ob) jobs.push_back(RbpJob{li, ob, -1});
            const size_t nw = (size_t)Kw * r.cout, nb = (size_t)r.cout * (L.bn_off >= 0 ? 3 : 1);
            for (size_t i = 0; i < nw; ++i) covered[(size_t)L.w_off + i] = 1;
            for (int o = 0; o < r.cout; ++o) covered[(size_t)L.b_off + o] = 1;
            if (L.bn_off >= 0) for (size_t i = 0; i < (size_t)2 * r.cout; ++i) covered[(size_t)L.bn_off + i] = 1;
            (void)nb;
        }
    }
    h->rbp_job0[3] = (int)jobs.size();
    // the downsampler (mz_dsbp_*): arena tensors per layer, one dW job per conv output channel
    std::vector<DsBpLayer> dlay;
    std::vector<DsDwJob> djobs;
    if (h->ds) {
        const DsPlan& D = h->dsplan;
        int o = 0, maxdt = 0;
        auto t = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
        dlay.resize(D.n);
        for (int i = 0; i < D.n; ++i) {
            const DsLayer& L = D.L[i];
            const int n = L.cout * L.Wo * L.Ho;
            dlay[i].x = i == 0 ? -1 : dlay[i - 1].y;
            dlay[i].y = t(n);
            dlay[i].z = L.kind == DS_CONV && L.bn ? t(n) : -1;
            dlay[i].res = L.res_add ? dlay[i - 1].x : -1;
            if (L.kind != DS_CONV) continue;
            maxdt = std::max(maxdt, n);
            const int K = L.kw * L.kh * L.cin;
            if (L.kw * L.kh + 3 > DS_DW_THREADS) return fail(h, "corrected learner: a downsampler conv has too many taps");
            for (int co = 0; co < L.cout; ++co)
                for (int ci = 0; ci < L.cin; ++ci) djobs.push_back(DsDwJob{i, co, ci});
            for (int e = 0; e < K * L.cout; ++e) covered[(size_t)L.woff + e] = 1;
            for (int co = 0; co < L.cout; ++co) covered[(size_t)L.boff + co] = 1;
            if (L.bn) for (int e = 0; e < 2 * L.cout; ++e) covered[(size_t)L.bnoff + e] = 1;
        }
        h->dsbp_dt = o;
        h->dsbp_arena = o + ((maxdt + 3) & ~3);
        h->dsbp_n_job = (int)djobs.size();
    }
    for (size_t i = 0; i < h->nflat; ++i)
        if (!covered[i]) return fail(h, "corrected learner: a parameter no gradient job covers");
    auto up = [&](auto** d, const auto& v) -> int {
        MZ_TRY(h, dalloc(h, d, v.size()));
        MZ_TRY(h, hipMemcpy(*d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice));
        return 0;
    };
    if (up(&h->d_rbp_apps, apps) || up(&h->d_rbp_heads, heads) || up(&h->d_rbp_layers, layers) ||
        up(&h->d_rbp_uses, uses) || up(&h->d_rbp_jobs, jobs) || up(&h->d_rbp_gzero, gz))
        return -1;
    if (h->ds && (up(&h->d_dsbp_lay, dlay) || up(&h->d_dsbp_jobs, djobs))) return -1;
    h->rbp_n_gzero = (int)gz.size();
    // Σθ² per job: the downsampler's jobs first (net 0), then mz_rbp_dw's
    MZ_TRY(h, dalloc(h, &h->d_rbp_sq, jobs.size() + djobs.size()));
    h->rbp_n_app = (int)apps.size(); h->rbp_n_head = (int)heads.size(); h->rbp_n_job = (int)jobs.size();
    h->rbp_arena = off; h->rbp_obs_t = obs_t; h->rbp_dt = (dtf + 3) & ~3; h->rbp_xs = (xsf + 3) & ~3;
    // a wave per 16x16 conv block of a pass (mz_rbp_sample), 4 to 12 waves
    h->rbp_threads = 64 * std::min(12, std::max(4, max_units));
    const size_t lds = (size_t)(h->rbp_dt * (1 + h->rbp_ring) + h->rbp_xs) * 4;
    if (lds > kLdsMax) return fail(h, "corrected learner: a conv's tensors exceed the LDS");
    // above the 64 KB default (e.g. 256 filters on the 6x7 board: ~86 KB)
    MZ_TRY(h, hipFuncSetAttribute((const void*)mz_rbp_sample, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    h->rbp_built = true;
    return 0;
}

static int rbp_grad(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, hipStream_t st) {
    const int B = b->batch_size, K = h->conf.num_unroll_steps;
    if (!h->rbp_built && build_rbp(h)) return -1;
    if (ensure_batch(h, B)) return -1;
    if (B > h->rbp_cap) {
        MZ_TRY(h, dalloc(h, &h->d_rbp_act, (size_t)B * h->rbp_arena));
        MZ_TRY(h, dalloc(h, &h->d_rbp_grad, (size_t)B * h->rbp_arena));
        MZ_TRY(h, dalloc(h, &h->d_rbp_terms, (size_t)B * (K + 1) * 3));
        h->rbp_cap = B;
    }
    if (h->ds && B > h->dsbp_cap) {
        MZ_TRY(h, dalloc(h, &h->d_dsbp_act, (size_t)B * h->dsbp_arena));
        MZ_TRY(h, dalloc(h, &h->d_dsbp_grad, (size_t)B * h->dsbp_arena));
        h->dsbp_cap = B;
    }
    DsBpParams DP;
    if (h->ds) {                                  // the downsampler's forward, its output the tail's input
        if (ensure_dsb(h, B)) return -1;
        DP.B = B; DP.arena = h->dsbp_arena; DP.bn_s = h->bn_s; DP.plan = h->d_dsplan; DP.lay = h->d_dsbp_lay;
        DP.flat = h->d_flat; DP.obs = b->observation; DP.act = h->d_dsbp_act; DP.grad = h->d_dsbp_grad;
        DP.out = h->d_dsb; DP.gout = h->d_rbp_grad; DP.gstride = h->rbp_arena; DP.goff = h->rbp_obs_t;
        DP.dt_off = h->dsbp_dt;
        hipLaunchKernelGGL(mz_dsbp_fwd, dim3(B), dim3(DS_THREADS), 0, st, DP);
    }
    if ((size_t)B * (size_t)std::max(1, K + 1) * (size_t)h->plane >= (1u << 20))
        return fail(h, "corrected learner: batch x unroll x board too large for the dW index");
    RbpParams Q;
    Q.B = B; Q.K = K; Q.A = h->A; Q.H = h->H; Q.P = h->plane; Q.Wb = h->rconf.observation_shape[0];
    Q.obs_feat = h->rin_feat; Q.arena = h->rbp_arena; Q.n_app = h->rbp_n_app; Q.n_head = h->rbp_n_head;
    Q.obs_t = h->rbp_obs_t; Q.intermediate_rewards = h->conf.intermediate_rewards; Q.nflat = (int)h->nflat;
    Q.dt_floats = h->rbp_dt; Q.xs_floats = h->rbp_xs; Q.gzero = h->d_rbp_gzero; Q.n_gzero = h->rbp_n_gzero;
    Q.apps = h->d_rbp_apps; Q.heads = h->d_rbp_heads;
    Q.act = h->d_rbp_act; Q.grad = h->d_rbp_grad; Q.flat = h->d_flat;
    Q.obs = h->ds ? h->d_dsb : b->observation; Q.actions = b->actions; Q.tv = b->target_values;
    Q.tr = b->target_rewards;
    Q.tp = b->target_policies; Q.gscale = b->gradient_scale; Q.weights = b->weights; Q.terms = h->d_rbp_terms;
    Q.pv = h->d_pv; Q.pp = h->d_pp; Q.pr = h->d_pr;
    Q.stamps = nullptr;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, 128)));
    Q.stamps = h->d_stamps;
#endif
    hipLaunchKernelGGL(mz_rbp_sample, dim3(B), dim3(h->rbp_threads),
                       (size_t)(h->rbp_dt * (1 + h->rbp_ring) + h->rbp_xs) * 4, st, Q);
    const int nds = h->ds ? h->dsbp_n_job : 0;
    if (h->ds) {                                  // ∂L/∂(downsampler output) is the arena's obs tensor
        hipLaunchKernelGGL(mz_dsbp_bwd, dim3(B), dim3(DS_THREADS), 0, st, DP);
        DsDwParams DW;
        DW.B = B; DW.arena = h->dsbp_arena; DW.n_job = nds; DW.bn_s = h->bn_s; DW.plan = h->d_dsplan;
        DW.lay = h->d_dsbp_lay; DW.jobs = h->d_dsbp_jobs; DW.obs = b->observation; DW.act = h->d_dsbp_act;
        DW.grad = h->d_dsbp_grad; DW.flat = h->d_flat; DW.out = grad_dev ? grad_dev : h->d_grad; DW.sq = h->d_rbp_sq;
        hipLaunchKernelGGL(mz_dsbp_dw, dim3(nds), dim3(DS_DW_THREADS), 0, st, DW);
    }
    RbpDwParams D;
    D.B = B; D.P = h->plane; D.Wb = h->rconf.observation_shape[0]; D.arena = h->rbp_arena;
    D.jobs = h->d_rbp_jobs; D.layers = h->d_rbp_layers; D.uses = h->d_rbp_uses;
    D.act = h->d_rbp_act; D.grad = h->d_rbp_grad; D.flat = h->d_flat;
    D.out = grad_dev ? grad_dev : h->d_grad; D.sq = h->d_rbp_sq + nds;
    hipLaunchKernelGGL(mz_rbp_dw, dim3(h->rbp_n_job), dim3(64 * RBP_DW_WAVES), 0, st, D);
    BpFoldParams F;
    F.B = B; F.K = K; F.terms = h->d_rbp_terms; F.gscale = b->gradient_scale; F.weights = b->weights;
    F.flat = h->d_flat; F.netoff = h->d_netoff; F.losses = losses_dev ? losses_dev : h->d_loss;
    F.sq = h->d_rbp_sq;
    for (int n = 0; n < 4; ++n) F.job0[n] = n == 0 ? 0 : h->rbp_job0[n] + nds;
    hipLaunchKernelGGL(mz_bp_fold, dim3(4), dim3(256), 0, st, F);
    MZ_TRY(h, hipGetLastError());
    h->last_lvariant = h->ds ? "mz_dsbp+mz_rbp_sample+mz_rbp_dw" : "mz_rbp_sample+mz_rbp_dw";
    return 0;
}

// corrected step: gradient (data term + 2θ) into grad_dev, losses, read-outs
static int bp_grad(mz_handle* h, const mz_batch* b, float* grad_dev, float* losses_dev, hipStream_t st) {
    if (h->kind == 1) return rbp_grad(h, b, grad_dev, losses_dev, st);
    const int B = b->batch_size, K = h->conf.num_unroll_steps;
    if (!h->bp_built && build_bp(h)) return -1;
    if (ensure_batch(h, B)) return -1;
    const int tiles = (B + 15) / 16;
    if (tiles > h->bp_tiles_cap) {
        MZ_TRY(h, dalloc(h, &h->d_bp_act, (size_t)tiles * h->bp_tile_floats));
        MZ_TRY(h, dalloc(h, &h->d_bp_grad, (size_t)tiles * h->bp_tile_floats));
        MZ_TRY(h, dalloc(h, &h->d_bp_terms, (size_t)tiles * 16 * (K + 1) * 3));
        h->bp_tiles_cap = tiles;
    }
    BpParams Q;
    Q.B = B; Q.K = K; Q.A = h->A; Q.H = h->H; Q.plane = h->plane; Q.obs_feat = h->obs_feat;
    Q.tile_floats = h->bp_tile_floats; Q.n_app = h->bp_n_app; Q.n_head = h->bp_n_head; Q.obs_t = h->bp_obs_t;
    Q.intermediate_rewards = h->conf.intermediate_rewards;
    Q.apps = h->d_bp_apps; Q.heads = h->d_bp_heads; Q.act = h->d_bp_act; Q.grad = h->d_bp_grad; Q.flat = h->d_flat;
    Q.obs = b->observation; Q.actions = b->actions; Q.tv = b->target_values; Q.tr = b->target_rewards;
    Q.tp = b->target_policies; Q.gscale = b->gradient_scale; Q.weights = b->weights; Q.terms = h->d_bp_terms;
    Q.pv = h->d_pv; Q.pp = h->d_pp; Q.pr = h->d_pr;
    Q.n_flev = h->bp_n_flev; Q.n_blev = h->bp_n_blev; Q.n_funit = h->bp_n_funit; Q.n_bunit = h->bp_n_bunit;
    Q.fsync = h->d_bp_fsync; Q.bsync = h->d_bp_bsync; Q.cache_floats = h->bp_cache_floats; Q.obs_s = h->bp_obs_s;
    static const bool no_warm = std::getenv("MZ_BP_NO_WARM") != nullptr;   // A/B only
    Q.nflat = no_warm ? 0 : (int)h->nflat;
    const size_t lv_lds = (size_t)Q.n_app * sizeof(BpApp) + (size_t)(Q.n_funit + Q.n_bunit) * sizeof(int2) +
                          (size_t)(2 * (Q.n_flev + Q.n_blev) + 8) * sizeof(int) + 16 + (size_t)Q.cache_floats * 4;
    Q.funits = h->d_bp_funits; Q.flev = h->d_bp_flev; Q.bunits = h->d_bp_bunits; Q.blev = h->d_bp_blev;
    Q.stamps = nullptr;
#ifdef MZ_STAMPS
    if (!h->d_stamps) MZ_TRY(h, dalloc(h, &h->d_stamps, (size_t)8 * std::max(h->max_games, 128)));
    Q.stamps = h->d_stamps;
#endif
    // the level schedule (default) or the one-application-per-barrier kernel
    // (MZ_BP_SEQ=1, the same bits: tests/test_corrected_learner_gpu.py)
    if (std::getenv("MZ_BP_SEQ")) hipLaunchKernelGGL(mz_bp_tile, dim3(tiles), dim3(256), 0, st, Q);
    else if (lv_lds <= kLdsMax)                   // (no BatchNorm layer: the kernel without its per-layer test)
        hipLaunchKernelGGL(h->hp.use_batch_norm ? mz_bp_tile_lv : mz_bp_tile_lv_nobn, dim3(tiles), dim3(BP_LV_THREADS),
                           lv_lds, st, Q);
    else return fail(h, "corrected learner: the level schedule exceeds the LDS");
    BpDwParams D;
    D.tiles = tiles; D.tile_floats = h->bp_tile_floats; D.n_job = h->bp_n_job; D.jobs = h->d_bp_jobs;
    D.layers = h->d_bp_layers; D.uses = h->d_bp_uses; D.act = h->d_bp_act; D.grad = h->d_bp_grad; D.flat = h->d_flat;
    D.out = grad_dev ? grad_dev : h->d_grad;
    D.sq = h->d_bp_sq;
    hipLaunchKernelGGL(mz_bp_dw, dim3(h->bp_n_job), dim3(64), 0, st, D);
    BpFoldParams F;
    F.B = B; F.K = K; F.terms = h->d_bp_terms; F.gscale = b->gradient_scale; F.weights = b->weights;
    F.flat = h->d_flat; F.netoff = h->d_netoff; F.losses = losses_dev ? losses_dev : h->d_loss;
    F.sq = h->d_bp_sq;
    for (int n = 0; n < 4; ++n) F.job0[n] = h->bp_job0[n];
    hipLaunchKernelGGL(mz_bp_fold, dim3(4), dim3(256), 0, st, F);
    MZ_TRY(h, hipGetLastError());
    return 0;
}

int mz_learner_set_mode(mz_handle* h, int mode) {
    if (!h) return -2;
    if (mode != MZ_LEARN_REF_SEMANTICS && mode != MZ_LEARN_CORRECTED) return fail(h, "unknown learner mode");
    h->learn_mode = mode;
    return 0;
}

int mz_learner_apply_dev(mz_handle* h, const float* grad_dev, float grad_scale, double eta, void* stream) {
    if (!h) return -2;
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    const float* g = grad_dev ? grad_dev : h->d_grad;
    hipLaunchKernelGGL(mz_adam_kernel, dim3(128), dim3(MZ_THREADS), 0, st, h->d_flat, h->d_m, h->d_v, g,
                       grad_scale, h->nflat, h->bp1, h->bp2, eta, h->d_Wp, h->d_Bp, h->d_inv_tile, h->d_sm_w,
                       h->d_sm_bias, h->d_inv_small);
    adam_advance(h);
    MZ_TRY(h, hipGetLastError());
    return 0;
}

int mz_learner_step(mz_handle* h, const mz_batch* b, double eta, float* losses_out) {
    if (!h || !b) return -2;
    const int B = b->batch_size, K = h->conf.num_unroll_steps, A = h->A;
    MZ_TRY(h, hipSetDevice(h->device));
    if (B < 1) return fail(h, "batch_size must be >= 1");
    if (ensure_batch(h, B)) return -1;
    MZ_SYNC(h);                  // `_dev` work on other streams first
    hipStream_t st = h->stream;
    MZ_TRY(h, hipMemcpyAsync(h->d_bobs, b->observation, (size_t)B * h->obs_feat * 4, hipMemcpyHostToDevice, st));
    MZ_TRY(h, hipMemcpyAsync(h->d_bact, b->actions, (size_t)B * (K + 1) * 4, hipMemcpyHostToDevice, st));
    MZ_TRY(h, hipMemcpyAsync(h->d_btv, b->target_values, (size_t)B * (K + 1) * 4, hipMemcpyHostToDevice, st));
    MZ_TRY(h, hipMemcpyAsync(h->d_btr, b->target_rewards, (size_t)B * (K + 1) * 4, hipMemcpyHostToDevice, st));
    MZ_TRY(h, hipMemcpyAsync(h->d_btp, b->target_policies, (size_t)B * (K + 1) * A * 4, hipMemcpyHostToDevice, st));
    MZ_TRY(h, hipMemcpyAsync(h->d_bgs, b->gradient_scale, (size_t)B * 4, hipMemcpyHostToDevice, st));
    if (b->weights) MZ_TRY(h, hipMemcpyAsync(h->d_bw, b->weights, (size_t)B * 4, hipMemcpyHostToDevice, st));
    mz_batch db = *b;
    db.observation = h->d_bobs; db.actions = h->d_bact; db.target_values = h->d_btv;
    db.target_rewards = h->d_btr; db.target_policies = h->d_btp; db.gradient_scale = h->d_bgs;
    db.weights = b->weights ? h->d_bw : nullptr;
    int rc = mz_learner_grad_dev(h, &db, h->d_grad, h->d_loss, st);
    if (rc) return rc;
    rc = mz_learner_apply_dev(h, h->d_grad, 1.0f, eta, st);
    if (rc) return rc;
    if (losses_out) MZ_TRY(h, hipMemcpyAsync(losses_out, h->d_loss, 6 * 4, hipMemcpyDeviceToHost, st));
    MZ_TRY(h, hipStreamSynchronize(st));
    return check_fault(h);
}

// the next (start, stop) event pair of the measurement list (mz_debug_kernel_time)
static int timing_events(mz_handle* h, hipEvent_t* e0, hipEvent_t* e1) {
    if (h->tev_used + 2 > h->tev.size())
        for (int i = 0; i < 2; ++i) {
            hipEvent_t e;
            MZ_TRY(h, hipEventCreate(&e));
            h->tev.push_back(e);
        }
    *e0 = h->tev[h->tev_used++]; *e1 = h->tev[h->tev_used++];
    return 0;
}

int mz_debug_kernel_time(mz_handle* h, double* total_ms, int* launches) {
    if (!h) return -2;
    MZ_TRY(h, hipSetDevice(h->device));
    double t = 0.0;
    for (size_t i = 0; i + 1 < h->tev_used; i += 2) {
        MZ_TRY(h, hipEventSynchronize(h->tev[i + 1]));
        float ms = 0.0f;
        MZ_TRY(h, hipEventElapsedTime(&ms, h->tev[i], h->tev[i + 1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = (int)(h->tev_used / 2);
    h->tev_used = 0;
    return 0;
}

int mz_debug_unroll(mz_handle* h, int B, float* values, float* policies, float* rewards) {
    if (!h) return -2;
    if (B < 0 || B > h->bcap) return fail(h, "B exceeds the last learner batch");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    const size_t n = (size_t)B * (h->conf.num_unroll_steps + 1);
    if (values) MZ_TRY(h, hipMemcpy(values, h->d_pv, n * 4, hipMemcpyDeviceToHost));
    if (policies) MZ_TRY(h, hipMemcpy(policies, h->d_pp, n * h->A * 4, hipMemcpyDeviceToHost));
    if (rewards) MZ_TRY(h, hipMemcpy(rewards, h->d_pr, n * 4, hipMemcpyDeviceToHost));
    return 0;
}

// Diagnostic: per-workgroup phase cycles of the last search (stamp build only).
int mz_debug_stamps(mz_handle* h, unsigned long long* out, int n_blocks) {
    if (!h) return -2;
#ifdef MZ_STAMPS
    if (!h->d_stamps) return fail(h, "no stamps recorded");
    MZ_SYNC(h);
    MZ_TRY(h, hipMemcpy(out, h->d_stamps, (size_t)n_blocks * 8 * 8, hipMemcpyDeviceToHost));
    return 0;
#else
    (void)out; (void)n_blocks;
    return fail(h, "libmz built without -DMZ_STAMPS");
#endif
}

const char* mz_search_variant(const mz_handle* h) {
    if (!h) return "";
    return h->last_variant.c_str();
}

const char* mz_learner_variant(const mz_handle* h) {
    if (!h) return "";
    return h->last_lvariant.c_str();
}

// ------------------------------------------------ device self-play + replay
}  // extern "C"

// ------------------------------------------------ checkpoint interface (mz_ckpt_iface.h)
static const char* kNetNames[3] = {"representation", "prediction", "dynamics"};

std::vector<MzParamDesc> mz_param_table(const mz_handle* h) {
    std::vector<MzParamDesc> t;
    for (int net = 0; net < 3; ++net) {
        int i = 0;
        auto add = [&](std::vector<int64_t> shp, size_t off) {
            size_t cnt = 1;
            for (int64_t d : shp) cnt *= (size_t)d;
            t.push_back(MzParamDesc{std::string(kNetNames[net]) + "." + std::to_string(i++), shp, off, cnt});
        };
        if (h->kind == 0) {                                   // Dense: W (out, in), b (out)
            for (const LayerSpec& L : h->layers) {
                if (L.net != net) continue;
                add({L.out, L.in}, L.flux_w);
                add({L.out}, L.flux_b);
                if (L.bn) { add({L.out}, L.flux_be); add({L.out}, L.flux_be + L.out); }   // BatchNorm β, γ
            }
        } else {                                              // Conv: W (kw,kh,cin,cout), b, BatchNorm β, γ
            size_t np = 0;
            if (net == MZ_NET_REPR && h->ds)                  // the downsampler's convs first (MeanPool: none)
                for (int i = 0; i < h->dsplan.n; ++i) {
                    const DsLayer& L = h->dsplan.L[i];
                    if (L.kind != DS_CONV) continue;
                    add({L.kw, L.kh, L.cin, L.cout}, h->flat_off[net] + L.woff);
                    add({L.cout}, h->flat_off[net] + L.boff);
                    if (L.bn) { add({L.cout}, h->flat_off[net] + L.bnoff); add({L.cout}, h->flat_off[net] + L.bnoff + L.cout); }
                }
            for (const RSpec& r : rn_specs(h->rconf, h->rhp, net, &np)) {
                const size_t base = h->flat_off[net] + (net == MZ_NET_REPR ? h->ds_n : 0);
                if (r.conv) {
                    add({r.kw, r.kh, r.cin, r.cout}, base + r.woff);
                    add({r.cout}, base + r.boff);
                    add({r.cout}, base + r.bnoff);
                    add({r.cout}, base + r.bnoff + r.cout);
                } else {
                    add({r.cout, r.cin}, base + r.woff);
                    add({r.cout}, base + r.boff);
                }
            }
        }
    }
    return t;
}

size_t mz_flat_count(const mz_handle* h) { return h->nflat; }

int mz_state_get(mz_handle* h, float* flat, float* m, float* v, double* beta_pow) {
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    if (flat) MZ_TRY(h, hipMemcpy(flat, h->d_flat, h->nflat * 4, hipMemcpyDeviceToHost));
    if (m) MZ_TRY(h, hipMemcpy(m, h->d_m, h->nflat * 4, hipMemcpyDeviceToHost));
    if (v) MZ_TRY(h, hipMemcpy(v, h->d_v, h->nflat * 4, hipMemcpyDeviceToHost));
    if (beta_pow) { beta_pow[0] = h->bp1; beta_pow[1] = h->bp2; }
    return 0;
}

int mz_state_set(mz_handle* h, const float* flat, const float* m, const float* v, const double* beta_pow) {
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    MZ_TRY(h, hipMemcpy(h->d_flat, flat, h->nflat * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_m, m, h->nflat * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_v, v, h->nflat * 4, hipMemcpyHostToDevice));
    h->bp1 = beta_pow[0]; h->bp2 = beta_pow[1];
    if (repack(h)) return -1;
    MZ_SYNC(h);
    return 0;
}

std::string mz_net_kind(const mz_handle* h) { return h->kind == 0 ? "fc" : "resnet"; }

std::string mz_describe(const mz_handle* h) {
    const mz_config& c = h->conf;
    std::string s = "{\"observation_shape\":[" + std::to_string(c.observation_shape[0]) + "," +
                    std::to_string(c.observation_shape[1]) + "," + std::to_string(c.observation_shape[2]) + "]" +
                    ",\"action_space_size\":" + std::to_string(c.action_space_size) +
                    ",\"stacked_observations\":" + std::to_string(c.stacked_observations) +
                    ",\"num_unroll_steps\":" + std::to_string(c.num_unroll_steps);
    if (h->kind == 0) {
        const mz_ffhp& p = h->hp;
        s += ",\"width_hidden\":" + std::to_string(p.width_hidden) +
             ",\"depth_representation\":" + std::to_string(p.depth_representation) +
             ",\"depth_prediction\":" + std::to_string(p.depth_prediction) +
             ",\"depth_dynamics\":" + std::to_string(p.depth_dynamics) +
             ",\"depth_policy\":" + std::to_string(p.depth_policy) + ",\"depth_value\":" + std::to_string(p.depth_value) +
             ",\"depth_reward\":" + std::to_string(p.depth_reward) +
             ",\"depth_state_head\":" + std::to_string(p.depth_state_head) +
             ",\"hidden_state_size\":" + std::to_string(p.hidden_state_size) +
             ",\"reward_activation\":" + std::to_string(p.reward_activation);
    } else {
        const mz_resnet_hp& p = h->rhp;
        s += ",\"num_blocks\":" + std::to_string(p.num_blocks) + ",\"num_filters\":" + std::to_string(p.num_filters) +
             ",\"conv_kernel_size\":[" + std::to_string(p.conv_kernel_size[0]) + "," +
             std::to_string(p.conv_kernel_size[1]) + "]" +
             ",\"num_first_head_filters\":" + std::to_string(p.num_first_head_filters) +
             ",\"num_second_head_filters\":" + std::to_string(p.num_second_head_filters) +
             ",\"depth_value\":" + std::to_string(p.depth_value) + ",\"width_hidden\":" + std::to_string(p.width_hidden) +
             ",\"downsample\":" + std::to_string(p.downsample) +
             ",\"reward_activation\":" + std::to_string(p.reward_activation);
    }
    return s + "}";
}

int mz_set_error(mz_handle* h, const std::string& msg) { return fail(h, msg); }

template <typename T>
static hipError_t spalloc(mz_handle* h, T** p, size_t n, bool zero = true) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T) + 16);
    if (e == hipSuccess) {
        h->sp_allocs.push_back(*p);
        if (zero) e = hipMemset(*p, 0, n * sizeof(T) + 16);
    }
    return e;
}

static int sp_alloc_hist(mz_handle* h, SpHist& r, size_t n) {
    const size_t T = (size_t)h->sp_T, A = (size_t)h->A;
    MZ_TRY(h, spalloc(h, &r.obs, n * T * h->sp_osz));
    MZ_TRY(h, spalloc(h, &r.act, n * T));
    MZ_TRY(h, spalloc(h, &r.rew, n * T));
    MZ_TRY(h, spalloc(h, &r.tp, n * T));
    MZ_TRY(h, spalloc(h, &r.cv, n * T * A));
    MZ_TRY(h, spalloc(h, &r.rv, n * T));
    MZ_TRY(h, spalloc(h, &r.len, n));
    MZ_TRY(h, spalloc(h, &r.prio, n * T));
    MZ_TRY(h, spalloc(h, &r.gprio, n));
    return 0;
}

static SpParams sp_params(mz_handle* h) {
    SpParams S;
    std::memset(&S, 0, sizeof(S));
    const mz_config& c = h->conf;
    S.G = h->sp_G; S.env = h->sp_env; S.W = c.observation_shape[0]; S.H = c.observation_shape[1];
    S.osz = h->sp_osz; S.P = h->plane; S.A = h->A; S.F = h->obs_feat; S.stacked = c.stacked_observations;
    S.T = h->sp_T; S.max_moves = c.max_moves;
    S.board = h->d_sp_board; S.player = h->d_sp_player; S.over = h->d_sp_over;
    S.frames = h->sp_frames; S.ekey = h->d_sp_ekey;
    S.hist = h->sp_hist; S.ring = h->sp_ring; S.cap = h->sp_cap; S.counters = h->d_sp_counters;
    S.obs = h->d_obs; S.legal = h->d_legal; S.tp = h->d_tp; S.cv = h->d_cv; S.rv = h->d_rv; S.act = h->d_act;
    S.done = h->d_sp_done; S.ring_pos = h->d_sp_rpos;
    S.eval = h->sp_eval; S.opponent = h->sp_opp; S.muzero_player = h->sp_mzp;
    S.seed = h->seed; S.eval_counts = h->d_eval;
    S.per = c.PER != 0; S.per_alpha = c.PER_alpha; S.td = c.td_steps; S.disc_pow = h->d_sp_dpow;
    return S;
}

extern "C" {

int mz_selfplay_init(mz_handle* h, int env_kind, int G, int replay_games) {
    if (!h) return -2;
    const mz_config& c = h->conf;
    const int W = c.observation_shape[0], H = c.observation_shape[1], C = c.observation_shape[2];
    if (env_kind == MZ_ENV_TICTACTOE) {
        if (W != 3 || H != 3 || C != 3 || h->A != 9) return fail(h, "TicTacToe needs observation_shape (3,3,3), 9 actions");
    } else if (env_kind == MZ_ENV_CONNECT4) {
        if (W != 6 || H != 7 || C != 3 || h->A != 7) return fail(h, "Connect4 needs observation_shape (6,7,3), 7 actions");
    } else if (env_kind == MZ_ENV_ATARI) {
        if (W != 84 || H != 84 || C != 4 || h->A != 18 || c.stacked_observations != 0)
            return fail(h, "the Atari-like env needs observation_shape (84,84,4), 18 actions, stacked_observations 0");
    } else {
        return fail(h, "unknown env_kind");
    }
    if (G < 1 || G > h->max_games) return fail(h, "G must be in 1..max_games");
    if (replay_games < G) return fail(h, "replay_games must be >= G (one move can finish every slot)");
    if (c.max_moves < 1) return fail(h, "max_moves must be >= 1");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    for (void* p : h->sp_allocs) (void)hipFree(p);
    h->sp_allocs.clear();
    h->rs_cap = 0;
    h->pf_cap = 0; h->pf_cur = 0; h->d_pf_hdr = nullptr; ++h->pf_epoch;
    h->sp_has_games = false;
    h->sp_reset_pending = false;
    h->tr_B = 0;                                // a new shard: mz_train_init again
    h->sp_env = env_kind; h->sp_G = G; h->sp_cap = replay_games;
    h->sp_T = c.max_moves + 1; h->sp_osz = W * H * C;
    h->sp_frames = 0;
    if (env_kind == MZ_ENV_ATARI) { h->sp_osz = W * H; h->sp_frames = C; }   // one frame per move
    MZ_TRY(h, spalloc(h, &h->d_sp_board, (size_t)G * h->sp_osz));
    MZ_TRY(h, spalloc(h, &h->d_sp_player, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_sp_over, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_sp_ekey, (size_t)G));
    if (sp_alloc_hist(h, h->sp_hist, (size_t)G)) return -1;
    if (sp_alloc_hist(h, h->sp_ring, (size_t)replay_games)) return -1;
    MZ_TRY(h, spalloc(h, &h->d_sp_counters, 4));
    MZ_TRY(h, spalloc(h, &h->d_sp_done, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_sp_rpos, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_sp_temp, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_sp_tgame, (size_t)G));
    MZ_TRY(h, spalloc(h, &h->d_eval, 4));
    MZ_TRY(h, spalloc(h, &h->d_per_cum, (size_t)h->sp_cap));
    MZ_TRY(h, spalloc(h, &h->d_per_p, (size_t)h->sp_cap));
    MZ_TRY(h, spalloc(h, &h->d_per_total, 1));
    h->sp_eval = 0; h->sp_opp = MZ_OPP_SELF; h->sp_mzp = 1;
    // f32(discount^n) as Julia's Float32^Int (≈ f32(pow(f64))), n = 0..td+1
    std::vector<float> dp(c.td_steps + 2);
    for (int n = 0; n < (int)dp.size(); ++n) dp[n] = (float)std::pow((double)c.discount, (double)n);
    MZ_TRY(h, spalloc(h, &h->d_sp_dpow, dp.size()));
    MZ_TRY(h, hipMemcpy(h->d_sp_dpow, dp.data(), dp.size() * 4, hipMemcpyHostToDevice));
    if (env_kind == MZ_ENV_ATARI) {
        // every slot: new game, its key and first frame drawn on the device at
        // the first mz_selfplay_move, keyed by the global game id game_offset +
        // slot that the move carries (ranks of a data-parallel job hold
        // different games, not copies of slot 0..G-1's)
        h->sp_reset_pending = true;
        return 0;
    }
    // every slot: new game (boards: empty plane set, player 1)
    std::vector<uint8_t> b((size_t)G * h->sp_osz, 0);
    const int cells = W * H;
    for (int g = 0; g < G; ++g)
        for (int k = 2 * cells; k < 3 * cells; ++k) b[(size_t)g * h->sp_osz + k] = 1;
    std::vector<int32_t> pl(G, 1);
    MZ_TRY(h, hipMemcpy(h->d_sp_board, b.data(), b.size(), hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_sp_player, pl.data(), (size_t)G * 4, hipMemcpyHostToDevice));
    return 0;
}

int mz_selfplay_move(mz_handle* h, uint32_t rng_step, uint32_t game_offset, float temperature, void* stream) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    SpParams S = sp_params(h);
    S.step = rng_step; S.game_offset = game_offset;
    // temperature_threshold (SelfPlay.jl:344-346): per-slot temperatures
    const bool thr = h->conf.temperature_threshold >= 0;
    S.temperature = temperature; S.temp_threshold = h->conf.temperature_threshold;
    S.temp_g = thr || h->sp_latch ? h->d_sp_temp : nullptr;
    S.tgame = h->sp_latch ? h->d_sp_tgame : nullptr;
    const int G = h->sp_G;
    const dim3 waves((G + 3) / 4);
    if (h->sp_reset_pending) {                      // the initial Atari-like games (mz_selfplay_init)
        SpParams R = S;
        R.reset_step = 0xFFFFFFFFu;
        hipLaunchKernelGGL(mz_sp_reset, waves, dim3(256), 0, st, R);
        MZ_TRY(h, hipGetLastError());
        h->sp_reset_pending = false;
    }
    hipLaunchKernelGGL(mz_sp_prepare, waves, dim3(256), 0, st, S);
    MZ_TRY(h, hipGetLastError());
    int rc = search_dev(h, G, h->d_obs, h->d_legal, h->d_tp, 1, rng_step, game_offset, temperature, h->d_cv,
                        h->d_rv, h->d_act, st, S.temp_g);
    if (rc) return rc;
    hipLaunchKernelGGL(mz_sp_commit, waves, dim3(256), 0, st, S);
    hipLaunchKernelGGL(mz_sp_order, dim3(1), dim3(1024), 0, st, S);
    hipLaunchKernelGGL(mz_sp_store, dim3(G), dim3(256), 0, st, S);
    MZ_TRY(h, hipGetLastError());
    return 0;
}

int mz_selfplay_mode(mz_handle* h, int mode, int opponent, int muzero_player) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (mode != MZ_SP_TRAIN && mode != MZ_SP_EVAL) return fail(h, "mode must be MZ_SP_TRAIN or MZ_SP_EVAL");
    if (opponent != MZ_OPP_SELF && opponent != MZ_OPP_RANDOM) return fail(h, "opponent must be MZ_OPP_SELF or MZ_OPP_RANDOM");
    if (muzero_player != 1 && muzero_player != 2) return fail(h, "muzero_player must be 1 or 2");
    h->sp_eval = mode == MZ_SP_EVAL; h->sp_opp = opponent; h->sp_mzp = muzero_player;
    return 0;
}

int mz_eval_results(mz_handle* h, int64_t* out4) {
    if (!h || !out4) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    long long c[4];
    MZ_TRY(h, hipMemcpy(c, h->d_eval, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out4[i] = c[i];
    return 0;
}

int mz_replay_counts(mz_handle* h, int64_t* counts, int32_t* games_in_buffer) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    long long c[3];
    MZ_TRY(h, hipMemcpy(c, h->d_sp_counters, sizeof(c), hipMemcpyDeviceToHost));
    if (counts) for (int i = 0; i < 3; ++i) counts[i] = c[i];
    if (games_in_buffer) *games_in_buffer = (int32_t)std::min<long long>(c[0], h->sp_cap);
    return 0;
}

int mz_replay_save_game(mz_handle* h, int32_t T, const uint8_t* obs, const int32_t* actions, const float* rewards,
                        const int32_t* to_play, const float* child_visits, const float* root_values) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (T < 1 || T > h->sp_T) return fail(h, "game length must be in 1..max_moves+1");
    if (!obs || !actions || !rewards || !to_play || !child_visits || !root_values) return fail(h, "null array");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    long long c[3];
    MZ_TRY(h, hipMemcpy(c, h->d_sp_counters, sizeof(c), hipMemcpyDeviceToHost));
    const long long num = c[0] + 1;
    const int slot = (int)((num - 1) % h->sp_cap);
    if (num > h->sp_cap) {                          // the FIFO evicts game num - cap (:156-160)
        int32_t old = 0;
        MZ_TRY(h, hipMemcpy(&old, h->sp_ring.len + slot, 4, hipMemcpyDeviceToHost));
        c[2] -= old;
    }
    c[0] = num; c[1] += T; c[2] += T;
    const size_t base = (size_t)slot * h->sp_T, A = (size_t)h->A;
    const SpHist& r = h->sp_ring;
    MZ_TRY(h, hipMemcpy(r.obs + base * h->sp_osz, obs, (size_t)T * h->sp_osz, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.act + base, actions, (size_t)T * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.rew + base, rewards, (size_t)T * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.tp + base, to_play, (size_t)T * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.cv + base * A, child_visits, (size_t)T * A * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.rv + base, root_values, (size_t)T * 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(r.len + slot, &T, 4, hipMemcpyHostToDevice));
    MZ_TRY(h, hipMemcpy(h->d_sp_counters, c, sizeof(c), hipMemcpyHostToDevice));
    if (h->conf.PER) {                              // initial priorities (:136-143)
        hipLaunchKernelGGL(mz_rp_per_init, dim3(1), dim3(64), 0, h->stream, h->sp_ring, slot, (int)T, h->sp_T,
                           h->conf.td_steps, (const float*)h->d_sp_dpow, h->conf.PER_alpha);
        MZ_TRY(h, hipGetLastError());
        MZ_SYNC(h);
    }
    return 0;
}

// get_batch parameters for B samples at learner step `step` into the
// engine's batch arrays (allocated on first use); batch = those arrays
static int rs_params(mz_handle* h, int32_t B, uint32_t step, hipStream_t st, RpSampleParams* Qo, mz_batch* batch,
                     bool prefetching = false) {
    if (!prefetching) ++h->pf_epoch;              // set 0 is about to be refilled: its header is stale
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (B < 1) return fail(h, "batch_size must be >= 1");
    if (!h->sp_has_games) {                       // sample_n_games needs a non-empty buffer
        long long played = 0;
        MZ_TRY(h, hipStreamSynchronize(st));
        MZ_TRY(h, hipMemcpy(&played, h->d_sp_counters, sizeof(played), hipMemcpyDeviceToHost));
        if (played == 0) return fail(h, "replay buffer is empty");
        h->sp_has_games = true;
    }
    const int K1 = h->conf.num_unroll_steps + 1, A = h->A;
    if (B > h->rs_cap) {
        MZ_TRY(h, spalloc(h, &h->d_rs_obs, (size_t)B * h->obs_feat, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_act, (size_t)B * K1, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_tv, (size_t)B * K1, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_tr, (size_t)B * K1, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_tp, (size_t)B * K1 * A, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_gs, (size_t)B, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_index, (size_t)B * 2, false));
        MZ_TRY(h, spalloc(h, &h->d_rs_w, (size_t)B, false));
        h->rs_cap = B;
        ++h->pf_epoch;
    }
    RpSampleParams Q;
    std::memset(&Q, 0, sizeof(Q));
    Q.B = B; Q.K = K1 - 1; Q.A = A; Q.osz = h->sp_osz; Q.P = h->plane; Q.F = h->obs_feat;
    Q.stacked = h->conf.stacked_observations; Q.T = h->sp_T; Q.td = h->conf.td_steps; Q.cap = h->sp_cap;
    Q.frames = h->sp_frames;
    Q.seed = h->seed; Q.step = step; Q.ring = h->sp_ring; Q.counters = h->d_sp_counters; Q.disc_pow = h->d_sp_dpow;
    Q.obs = h->d_rs_obs; Q.actions = h->d_rs_act; Q.tv = h->d_rs_tv; Q.tr = h->d_rs_tr; Q.tpol = h->d_rs_tp;
    Q.gscale = h->d_rs_gs; Q.index = h->d_rs_index;
    Q.per = h->conf.PER != 0;
    if (Q.per) {                                  // game probabilities of the held games (:91-99)
        Q.per_cum = h->d_per_cum; Q.per_p = h->d_per_p; Q.per_total = h->d_per_total; Q.weights = h->d_rs_w;
        hipLaunchKernelGGL(mz_rp_per_prep, dim3(1), dim3(64), 0, st, h->sp_ring, (const long long*)h->d_sp_counters,
                           h->sp_cap, h->d_per_cum, h->d_per_p, h->d_per_total);
        MZ_TRY(h, hipGetLastError());
    }
    *Qo = Q;
    batch->batch_size = B;
    batch->observation = h->d_rs_obs; batch->actions = h->d_rs_act; batch->target_values = h->d_rs_tv;
    batch->target_rewards = h->d_rs_tr; batch->target_policies = h->d_rs_tp; batch->gradient_scale = h->d_rs_gs;
    batch->weights = Q.per ? h->d_rs_w : nullptr;
    return 0;
}

// PER: weight_batch ./= maximum(weight_batch) after the sampling launch
static int per_norm(mz_handle* h, int B, hipStream_t st) {
    if (!h->conf.PER) return 0;
    hipLaunchKernelGGL(mz_rp_per_norm, dim3(1), dim3(256), 0, st, h->d_rs_w, B);
    MZ_TRY(h, hipGetLastError());
    return 0;
}

// PER: update_priorities! of the last sampled batch from the last unroll's values
static int per_update(mz_handle* h, int B, hipStream_t st) {
    if (!h->conf.PER) return 0;
    hipLaunchKernelGGL(mz_rp_per_update, dim3(1), dim3(64), 0, st, h->sp_ring, (const long long*)h->d_sp_counters,
                       h->sp_cap, h->sp_T, B, h->conf.num_unroll_steps, h->conf.PER_alpha, h->d_rs_index, h->d_pv,
                       h->d_rs_tv);
    MZ_TRY(h, hipGetLastError());
    return 0;
}

int mz_replay_sample(mz_handle* h, int32_t B, uint32_t step, mz_batch* batch, int32_t* index_batch, void* stream) {
    if (!h || !batch) return -2;
    MZ_TRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    RpSampleParams Q;
    if (rs_params(h, B, step, st, &Q, batch)) return -1;
    hipLaunchKernelGGL(mz_rp_sample, dim3((B + 3) / 4), dim3(256), 0, st, Q);
    MZ_TRY(h, hipGetLastError());
    if (per_norm(h, B, st)) return -1;
    h->rs_last_B = B;
    if (index_batch) {
        MZ_TRY(h, hipMemcpyAsync(index_batch, h->d_rs_index, (size_t)B * 8, hipMemcpyDeviceToHost, st));
        MZ_TRY(h, hipStreamSynchronize(st));
    }
    return 0;
}

// the second batch set and the two headers of the get_batch prefetch
static int ensure_pf(mz_handle* h, int B) {
    if (B <= h->pf_cap && h->d_pf_hdr) return 0;
    const int K1 = h->conf.num_unroll_steps + 1, A = h->A;
    MZ_TRY(h, spalloc(h, &h->d_rs2_obs, (size_t)B * h->obs_feat, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_act, (size_t)B * K1, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_tv, (size_t)B * K1, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_tr, (size_t)B * K1, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_tp, (size_t)B * K1 * A, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_gs, (size_t)B, false));
    MZ_TRY(h, spalloc(h, &h->d_rs2_index, (size_t)B * 2, false));
    if (!h->d_pf_hdr) MZ_TRY(h, spalloc(h, &h->d_pf_hdr, 8));   // zeroed: matches no epoch
    h->pf_cap = B;
    ++h->pf_epoch;
    return 0;
}

// point the sampler's outputs and the batch at batch set s (0: d_rs_*, 1: d_rs2_*)
static void pf_set(mz_handle* h, int s, RpSampleParams* Q, mz_batch* b) {
    Q->obs = s ? h->d_rs2_obs : h->d_rs_obs; Q->actions = s ? h->d_rs2_act : h->d_rs_act;
    Q->tv = s ? h->d_rs2_tv : h->d_rs_tv; Q->tr = s ? h->d_rs2_tr : h->d_rs_tr;
    Q->tpol = s ? h->d_rs2_tp : h->d_rs_tp; Q->gscale = s ? h->d_rs2_gs : h->d_rs_gs;
    Q->index = s ? h->d_rs2_index : h->d_rs_index;
    if (b) {
        b->observation = Q->obs; b->actions = Q->actions; b->target_values = Q->tv;
        b->target_rewards = Q->tr; b->target_policies = Q->tpol; b->gradient_scale = Q->gscale;
    }
}

// Learner iteration on a batch drawn from this GPU's replay shard
// (get_batch + learning!, ReplayBuffer.jl:188-217, Learning.jl:327-404) with
// the sampling fused into the FC unroll kernel: results are those of
// mz_replay_sample(step) + mz_learner_grad_dev (+ mz_learner_apply_dev with
// grad_scale 1 for mz_learner_train_dev, whose ADAM update is fused into the
// loss kernel: one GPU, no gradient exchange).
static int learner_sampled(mz_handle* h, int32_t B, uint32_t step, float* grad_dev, float* losses_dev,
                           hipStream_t st, bool train, double eta) {
    MZ_TRY(h, hipSetDevice(h->device));
    RpSampleParams Q;
    mz_batch b;
    const int ti = small_unroll_ti(h, B);
    const bool fused = train && ti >= 0 && !h->conf.PER && h->A <= 16 && h->d_sm_w2 && h->kind != 1 &&
                       h->learn_mode != MZ_LEARN_CORRECTED && !std::getenv("MZ_LEARN_2LAUNCH");
    const bool pf = fused && !std::getenv("MZ_NO_BATCH_PREFETCH");
    if (rs_params(h, B, step, st, &Q, &b, pf)) return -1;
    if (ensure_batch(h, B)) return -1;
    if (pf && ensure_pf(h, B)) return -1;
    h->rs_last_B = B;
    if (h->learn_mode == MZ_LEARN_CORRECTED) {     // sample, backprop, (ADAM)
        hipLaunchKernelGGL(mz_rp_sample, dim3((B + 3) / 4), dim3(256), 0, st, Q);
        MZ_TRY(h, hipGetLastError());
        if (per_norm(h, B, st)) return -1;
        if (bp_grad(h, &b, train ? nullptr : grad_dev, losses_dev, st)) return -1;
        if (per_update(h, B, st)) return -1;                       // Learning.jl:400-404
        return train ? mz_learner_apply_dev(h, nullptr, 1.0f, eta, st) : 0;
    }
    if (h->kind == 1) {                             // ResNet: sample, then the network unroll
        if (h->conf.PER || h->ds) {                 // (else the sample is drawn inside the unroll launch)
            hipLaunchKernelGGL(mz_rp_sample, dim3((B + 3) / 4), dim3(256), 0, st, Q);
            MZ_TRY(h, hipGetLastError());
            if (per_norm(h, B, st)) return -1;
        }
        // one GPU: ADAM fused into the loss / Σθ² kernel (as the FC path)
        if (rlearner_grad(h, &b, train ? nullptr : grad_dev, losses_dev, st, train, eta,
                          h->conf.PER || h->ds ? nullptr : &Q)) return -1;
        return per_update(h, B, st);                               // Learning.jl:400-404
    }
    if (fused) {
        // one launch: unroll + losses ‖ Σθ² + ADAM into the second image set, then swap the sets;
        // with the prefetch, plus step + 1's get_batch into the other batch set
        const int cur = pf ? h->pf_cur : 0;
        RpSampleParams Qn = Q;
        if (pf) {
            pf_set(h, cur, &Q, &b);
            pf_set(h, 1 - cur, &Qn, nullptr);
            Qn.step = step + 1;
        }
        SmallUnrollParams U;
        if (small_unroll_params(h, &b, ti, &Q, &U)) return -1;
        U.pf_hdr = pf ? h->d_pf_hdr + 4 * cur : nullptr;
        U.pf_epoch = h->pf_epoch;
        LearnParams L;
        L.pf_nb = pf ? (B + SM_THREADS / 64 - 1) / (SM_THREADS / 64) : 0;
        L.pfq = Qn;
        L.pf_hdr_next = pf ? h->d_pf_hdr + 4 * (1 - cur) : nullptr;
        L.pf_epoch = h->pf_epoch;
        L.nU = (B + ti) / (ti + 1);
        L.tv = b.target_values; L.tp = b.target_policies; L.gscale = b.gradient_scale;
        L.terms = h->d_lterm; L.flat = h->d_flat; L.netoff = h->d_netoff; L.part = h->d_sq; L.counter = h->d_counter;
        L.out = losses_dev ? losses_dev : h->d_loss;
        L.ad = LgAdam{1, h->d_m, h->d_v, h->bp1, h->bp2, eta, h->d_Wp2, h->d_Bp2, h->d_inv_tile, h->d_sm_w2,
                      h->d_sm_bias2, h->d_inv_small};
        // MZ_LEARN_XCD=1: the unroll workgroups on one XCD (their weight image fetched into one L2):
        // PMC 3.79 MB per launch instead of 6.41 MB, but 31.4 k instead of 33.9 k steps/s (the 8·nU
        // grid and one L2 serving 32 workgroups; tools/ab_learn_xcd.sh, tools/pmc_learn_xcd.sh)
        const int roles = L.nU + LEARN_L2_GROUPS + L.pf_nb;
        static const bool xcd = std::getenv("MZ_LEARN_XCD") != nullptr;
        L.xcd = xcd && L.nU <= h->n_cu / 8 && 8 * L.nU >= roles;
        void* args[] = {&U, &L};
        MZ_TRY(h, hipLaunchKernel(h->sm_bn ? (ti == 0 ? (const void*)mz_learn_small1_bn : (const void*)mz_learn_small2_bn)
                                           : (ti == 0 ? (const void*)mz_learn_small1 : (const void*)mz_learn_small2),
                                  dim3(L.xcd ? 8 * L.nU : roles), dim3(SM_THREADS), args,
                                  unroll_small_lds(h, ti), st));
        if (pf) h->pf_cur = 1 - cur;
        h->last_lvariant = ti == 0 ? "mz_learn_small1" : "mz_learn_small2";
        std::swap(h->d_Wp, h->d_Wp2); std::swap(h->d_Bp, h->d_Bp2);
        std::swap(h->d_sm_w, h->d_sm_w2); std::swap(h->d_sm_bias, h->d_sm_bias2);
        adam_advance(h);
        return 0;
    }
    if (fc_unroll(h, &b, st, &Q)) return -1;
    if (per_norm(h, B, st)) return -1;
    if (learner_losses(h, &b, grad_dev, losses_dev, st, h->lay.v_act, h->lay.r_act, train, eta)) return -1;
    return per_update(h, B, st);                                   // Learning.jl:400-404
}

int mz_replay_update_priorities(mz_handle* h, void* stream) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (!h->conf.PER) return fail(h, "PER is off in the config");
    if (h->rs_last_B <= 0) return fail(h, "no batch sampled yet");
    MZ_TRY(h, hipSetDevice(h->device));
    return per_update(h, h->rs_last_B, stream ? (hipStream_t)stream : h->stream);
}

int mz_replay_get_priorities(mz_handle* h, int32_t i, float* priorities, float* game_priority) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    long long played = 0;
    MZ_TRY(h, hipMemcpy(&played, h->d_sp_counters, sizeof(played), hipMemcpyDeviceToHost));
    const long long n = std::min<long long>(played, h->sp_cap);
    if (i < 0 || i >= n) return fail(h, "game index out of range");
    const int slot = (int)((played - n + i) % h->sp_cap);
    int32_t T = 0;
    MZ_TRY(h, hipMemcpy(&T, h->sp_ring.len + slot, 4, hipMemcpyDeviceToHost));
    if (priorities)
        MZ_TRY(h, hipMemcpy(priorities, h->sp_ring.prio + (size_t)slot * h->sp_T, (size_t)T * 4, hipMemcpyDeviceToHost));
    if (game_priority) MZ_TRY(h, hipMemcpy(game_priority, h->sp_ring.gprio + slot, 4, hipMemcpyDeviceToHost));
    return 0;
}

int mz_learner_grad_sampled_dev(mz_handle* h, int32_t B, uint32_t step, float* grad_dev, float* losses_dev,
                                void* stream) {
    if (!h) return -2;
    return learner_sampled(h, B, step, grad_dev, losses_dev, stream ? (hipStream_t)stream : h->stream, false, 0.0);
}

// ---- data-parallel learner over RCCL through the C ABI
#define MZ_DP_ID_BYTES 128   // sizeof(ncclUniqueId)
int mz_dp_unique_id(uint8_t* id) {
    if (!id) return -2;
    if (!rccl().ok) return -1;
    return rccl().get_id(id) == 0 ? 0 : -1;
}

int mz_dp_init(mz_handle* h, int rank, int world, const uint8_t* id) {
    if (!h || !id) return -2;
    if (world < 1 || rank < 0 || rank >= world) return fail(h, "rank / world out of range");
    if (!rccl().ok) return fail(h, "librccl.so.1 not found");
    MZ_TRY(h, hipSetDevice(h->device));
    dp_destroy(h);
    RcclId v;
    std::memcpy(v.b, id, MZ_DP_ID_BYTES);
    void* comm = nullptr;
    const int rc = rccl().init_rank(&comm, world, v, rank);
    if (rc != 0) return fail(h, std::string("ncclCommInitRank: ") + (rccl().err ? rccl().err(rc) : "error"));
    h->dp_comm = comm; h->dp_world = world; h->dp_rank = rank;
    return 0;
}

int mz_dp_allreduce(mz_handle* h, float* grad_dev, void* stream) {
    if (!h) return -2;
    if (!h->dp_comm) return fail(h, "mz_dp_init first");
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    float* g = grad_dev ? grad_dev : h->d_grad;
    // ncclFloat32 = 7, ncclSum = 0
    const int rc = rccl().allreduce(g, g, h->nflat, 7, 0, h->dp_comm, st);
    if (rc != 0) return fail(h, std::string("ncclAllReduce: ") + (rccl().err ? rccl().err(rc) : "error"));
    return 0;
}

int mz_learner_train_dp(mz_handle* h, int32_t B, uint32_t step, double eta, float* losses_dev, void* stream) {
    if (!h) return -2;
    if (!h->dp_comm) return fail(h, "mz_dp_init first");
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    if (learner_sampled(h, B, step, nullptr, losses_dev, st, false, 0.0)) return -1;
    if (mz_dp_allreduce(h, nullptr, st)) return -1;
    return mz_learner_apply_dev(h, nullptr, 1.0f / (float)h->dp_world, eta, st);
}

int mz_learner_train_dev(mz_handle* h, int32_t B, uint32_t step, double eta, float* losses_dev, void* stream) {
    if (!h) return -2;
    return learner_sampled(h, B, step, nullptr, losses_dev, stream ? (hipStream_t)stream : h->stream, true, eta);
}

// ---- L consecutive ref_semantics learner steps (ChainParams, mz_small_params.h;
// Learning.jl:327-404 with get_batch keyed by the step, Q11).  The L steps run
// as chunks of up to MZ_MULTI_MAX steps, each one chain launch (the ADAM
// iterations) and unroll launches of up to MZ_MULTI_UNROLL steps, in stream
// order (32-step chains: the chain's fixed costs over twice the steps).  (Measured: the next
// sub-chunk's chain on a second stream, ordered by events, beside the unroll
// launch — 228.8 k vs 279.5 k steps/s at L = 64, 114.6 k vs ~170 k at L = 8:
// the cross-stream event waits cost more than the chain they hide.)
static bool multi_ok(const mz_handle* h) {
    return h->kind == 0 && h->learn_mode == MZ_LEARN_REF_SEMANTICS && !h->conf.PER && h->small_ok && h->A <= 16 &&
           h->d_sm_w2 && !std::getenv("MZ_NO_MULTI");
}
// Sub-chunk length Ls and T per workgroup for L steps of B samples: one sample
// per workgroup while the L·B workgroups fit one per CU; else two, with as
// many steps per sub-chunk as keep one workgroup per CU (16 at B = 32)
static int multi_plan(const mz_handle* h, int B, int L, int* Ls) {
    static const int force = std::getenv("MZ_MULTI_T") ? std::atoi(std::getenv("MZ_MULTI_T")) : 0;   // tests / A/B
    static const int ls_env = std::getenv("MZ_MULTI_LS") ? std::atoi(std::getenv("MZ_MULTI_LS")) : 0;
    int ti;
    // T = 4 (round 6) when the call has the steps to fill the chip with 4 samples per workgroup
    // (twice the steps per unroll launch as T = 2 for about 1.1x a stage's cost); T = 2 when L·B
    // exceeds the CUs; T = 1 below
    const int nU4 = (B + 3) / 4;
    if ((force == 1 || force == 2 || force == 4) && small_unroll_fits(h, force == 4 ? 2 : force - 1))
        ti = force == 4 ? 2 : force - 1;
    else if (!force && (size_t)L * B <= (size_t)h->n_cu && small_unroll_fits(h, 0)) ti = 0;
    else if (!force && L >= std::min(MZ_MULTI_MAX, h->n_cu / nU4) && (size_t)L * nU4 >= (size_t)h->n_cu &&
             small_unroll_fits(h, 2) && !std::getenv("MZ_MULTI_NO_T4")) ti = 2;
    else if (small_unroll_fits(h, 1)) ti = 1;
    else if (small_unroll_fits(h, 0)) ti = 0;
    else return -1;
    const int T = ti == 2 ? 4 : ti + 1, nU = (B + T - 1) / T;
    int ls = std::max(1, std::min(ti == 2 ? MZ_MULTI_MAX : MZ_MULTI_UNROLL, h->n_cu / nU));
    if (ls_env > 0) ls = std::min(MZ_MULTI_MAX, ls_env);          // (A/B: more than one workgroup per CU)
    *Ls = std::min(ls, L);
    return ti;
}
static int ensure_multi(mz_handle* h, int B, int L) {
    if (h->kind == 1 && !h->d_tbank_w) {
        // the ResNet image bank: 2 halves of MZ_MULTI_MAX copies of the MFMA image (positions no parameter
        // maps to as in the engine's image), the flat bank (θ of each step)
        const size_t nw = h->packed_w_n, nb = std::max<size_t>(h->packed_b_n, 1);
        MZ_TRY(h, dalloc(h, &h->d_tbank_w, (size_t)2 * MZ_MULTI_MAX * nw));
        MZ_TRY(h, dalloc(h, &h->d_tbank_b, (size_t)2 * MZ_MULTI_MAX * nb));
        MZ_TRY(h, dalloc(h, &h->d_fbank, (size_t)2 * MZ_MULTI_MAX * fbank_stride(h)));
        for (int i = 0; i < 2 * MZ_MULTI_MAX; ++i) {
            MZ_TRY(h, hipMemcpy(h->d_tbank_w + (size_t)i * nw, h->d_Wp, nw * 4, hipMemcpyDeviceToDevice));
            if (h->packed_b_n)
                MZ_TRY(h, hipMemcpy(h->d_tbank_b + (size_t)i * nb, h->d_Bp, nb * 4, hipMemcpyDeviceToDevice));
        }
    }
    if (h->kind != 1 && !h->d_bank_w) {
        // two halves of MZ_MULTI_MAX images: sub-chunk k writes half k mod 2 (a chain launch
        // never writes the images an unroll launch still in flight reads)
        MZ_TRY(h, dalloc(h, &h->d_bank_w, (size_t)2 * MZ_MULTI_MAX * h->sm_w_n));
        MZ_TRY(h, dalloc(h, &h->d_bank_b, (size_t)2 * MZ_MULTI_MAX * h->sm_b_n));
        // the positions no parameter maps to (zero chunks, unused rows) as in the
        // engine's images; every mapped position is rewritten by each chain launch
        for (int i = 0; i < 2 * MZ_MULTI_MAX; ++i) {
            MZ_TRY(h, hipMemcpy(h->d_bank_w + (size_t)i * h->sm_w_n, h->d_sm_w, h->sm_w_n * 4, hipMemcpyDeviceToDevice));
            MZ_TRY(h, hipMemcpy(h->d_bank_b + (size_t)i * h->sm_b_n, h->d_sm_bias, h->sm_b_n * 4,
                                hipMemcpyDeviceToDevice));
        }
    }
    // per-step scratch (batches, read-outs, loss terms, partials) is a ring of at most 2·MZ_MULTI_MAX
    // steps (slot = step mod R, R = the largest multiple of the chain length Lc <= 2·MZ_MULTI_MAX, so a
    // chain launch's steps and an unroll launch's steps are contiguous, and a chain launch that reuses
    // an earlier launch's slots runs after its unrolls in stream order); on growth the old arrays are
    // freed after the device drains
    L = std::min(L, 2 * MZ_MULTI_MAX);
    if (B <= h->ml_cap && L <= h->ml_cap_L) return 0;
    const int cb = std::max(B, h->ml_cap), cl = std::max(L, h->ml_cap_L);
    if (h->ml_cap) {
        MZ_TRY(h, hipDeviceSynchronize());
        void* olds[] = {h->d_ml_obs, h->d_ml_act, h->d_ml_tv, h->d_ml_tr, h->d_ml_tp, h->d_ml_gs, h->d_ml_index,
                        h->d_ml_pv, h->d_ml_pp, h->d_ml_pr, h->d_ml_terms, h->d_ml_part, h->d_ml_cnt, h->d_ml_out,
                        h->d_ml_hs, h->d_ml_ts, h->d_ml_prog, h->d_ml_dsb};
        for (void* o : olds) if (o && dfree(h, o)) return -1;
        h->d_ml_hs = h->d_ml_ts = h->d_ml_dsb = nullptr;
        h->d_ml_prog = nullptr;
    }
    const size_t K1 = (size_t)h->conf.num_unroll_steps + 1, A = (size_t)h->A, n = (size_t)cl * cb;
    MZ_TRY(h, dalloc(h, &h->d_ml_obs, n * h->obs_feat));
    MZ_TRY(h, dalloc(h, &h->d_ml_act, n * K1)); MZ_TRY(h, dalloc(h, &h->d_ml_tv, n * K1));
    MZ_TRY(h, dalloc(h, &h->d_ml_tr, n * K1)); MZ_TRY(h, dalloc(h, &h->d_ml_tp, n * K1 * A));
    MZ_TRY(h, dalloc(h, &h->d_ml_gs, n)); MZ_TRY(h, dalloc(h, &h->d_ml_index, 2 * n));
    MZ_TRY(h, dalloc(h, &h->d_ml_pv, n * K1)); MZ_TRY(h, dalloc(h, &h->d_ml_pp, n * K1 * A));
    MZ_TRY(h, dalloc(h, &h->d_ml_pr, n * K1)); MZ_TRY(h, dalloc(h, &h->d_ml_terms, 2 * n * K1));
    MZ_TRY(h, dalloc(h, &h->d_ml_part, (size_t)cl * 3 * MZ_L2_BLOCKS));
    MZ_TRY(h, dalloc(h, &h->d_ml_cnt, (size_t)cl * MZ_MULTI_CNT_STRIDE));
    MZ_TRY(h, hipMemset(h->d_ml_cnt, 0, (size_t)cl * MZ_MULTI_CNT_STRIDE * 4));
    MZ_TRY(h, dalloc(h, &h->d_ml_out, (size_t)cl * 8));
    if (h->kind == 1) {
        const size_t KH = (size_t)std::max(h->conf.num_unroll_steps, 1);
        MZ_TRY(h, dalloc(h, &h->d_ml_hs, n * KH * h->H)); MZ_TRY(h, dalloc(h, &h->d_ml_ts, n * KH * h->H));
        MZ_TRY(h, dalloc(h, &h->d_ml_prog, n));
        MZ_TRY(h, hipMemset(h->d_ml_prog, 0, n * sizeof(unsigned long long)));
        h->ml_prog_epoch = 0;
        if (h->ds) MZ_TRY(h, dalloc(h, &h->d_ml_dsb, n * h->rin_feat));
    }
    h->ml_cap = cb; h->ml_cap_L = cl;
    return 0;
}

// ResNet nets (ref_semantics, no PER): per sub-chunk of Ls steps, the chain launch (ADAM
// iterations into the MFMA image bank and the flat bank, Σθ² per step, the Ls batches), the
// downsampler over the Ls·B observations (Atari), the unroll launch(es) of rlearner_grad's
// form with the steps on gridDim.z (the fused form: step-major chain blocks, then the items;
// RUnrollParams.ms) and one loss launch of Ls·nlb blocks
static bool rmulti_ok(const mz_handle* h) {
    return h->kind == 1 && h->learn_mode == MZ_LEARN_REF_SEMANTICS && !h->conf.PER && !std::getenv("MZ_NO_MULTI") &&
           !std::getenv("MZ_RUNROLL_FUSED");
}
static int ensure_multi(mz_handle* h, int B, int L);
// θ after up to two given steps, copied out by the chain launch that computes them (mz_train_run:
// the actors' and the queued sets at refresh steps inside one learner chunk)
struct MultiCap {
    int64_t t[2];                                   // absolute learner steps (< 0: none)
    float* dst[2];                                  // nflat floats each
    const mz_handle::WSet* img0;                    // NULL or set 0's search images, written by the chain too
    bool* imaged0;                                  // set when a chain launch wrote them
};
// mz_learn_chain's helper workgroups (ChainParams::nh) for the nets with more parameters than one pass
// of the slices (MZ_CHAIN_HELP=0: off, A/B).  Measured (tools/gpu_r06t.sh): FC 32.1 -> 24.8 us per
// 32-step chain, ResNet configs[2] 63.3 -> 44.2 us.  Returns the helper count.
static int chain_helpers(mz_handle* h, ChainParams& C) {
    static const char* env = std::getenv("MZ_CHAIN_HELP");
    const size_t stride = (size_t)MZ_L2_BLOCKS * MZ_THREADS;
    int nht = 0;
    size_t hx_n = 0;
    for (int n = 0; n < 3; ++n) {
        const size_t c = h->nparams[n];
        C.nh[n] = c > stride ? (int)((c - stride + MZ_THREADS - 1) / MZ_THREADS) : 0;
        C.hoff[n] = hx_n;
        hx_n += c > stride ? c : 0;
        nht += C.nh[n];
    }
    const bool on = nht > 0 && (!env || std::atoi(env) != 0);
    if (!on) {
        C.nh[0] = C.nh[1] = C.nh[2] = 0;
        return 0;
    }
    if (!h->d_chcnt) {
        MZ_TRY(h, dalloc(h, &h->d_chx, (size_t)MZ_MULTI_MAX * hx_n));
        MZ_TRY(h, dalloc(h, &h->d_chcnt, (size_t)3 * MZ_L2_BLOCKS));
        MZ_TRY(h, hipMemset(h->d_chcnt, 0, (size_t)3 * MZ_L2_BLOCKS * sizeof(unsigned long long)));
    }
    C.hx = h->d_chx; C.hx_n = hx_n; C.hcnt = h->d_chcnt;
    return nht;
}
static void set_caps(ChainParams& C, const MultiCap* cap, int64_t first, int nc) {
    for (int j = 0; j < 2; ++j) {
        const bool in = cap && cap->t[j] >= first && cap->t[j] < first + nc;
        C.cap_i[j] = in ? (int)(cap->t[j] - first) : -1;
        C.cap_dst[j] = in ? cap->dst[j] : nullptr;
    }
    if (C.cap_i[0] >= 0 && cap->img0) {
        C.cap_img[0] = cap->img0->Wp; C.cap_img[1] = cap->img0->Bp;
        C.cap_img[2] = cap->img0->smw; C.cap_img[3] = cap->img0->smb;
        if (cap->imaged0) *cap->imaged0 = true;
    }
}
static int rlearner_multi(mz_handle* h, int32_t B, uint32_t step0, int32_t L, const double* eta, float* losses_dev,
                          float* theta_dev, hipStream_t st, float* out_last, const MultiCap* cap) {
    RpSampleParams Q;
    mz_batch b;
    if (rs_params(h, B, step0, st, &Q, &b, true)) return -1;
    if (ensure_batch(h, B) || ensure_multi(h, B, L)) return -1;
    static const int ls_env = std::getenv("MZ_MULTI_LS") ? std::atoi(std::getenv("MZ_MULTI_LS")) : 0;
    const int Ls = std::min(L, ls_env > 0 ? std::min(MZ_MULTI_UNROLL, ls_env) : MZ_MULTI_UNROLL);
    const int K = h->conf.num_unroll_steps, KH = std::max(K, 1), A = h->A;
    const size_t K1 = (size_t)K + 1;
    const size_t s_obs = (size_t)B * h->obs_feat, s_k1 = (size_t)B * K1, s_tp = (size_t)B * K1 * A;
    const size_t nw = h->packed_w_n, nb = std::max<size_t>(h->packed_b_n, 1);
    Q.obs = h->d_ml_obs; Q.actions = h->d_ml_act; Q.tv = h->d_ml_tv; Q.tr = h->d_ml_tr; Q.tpol = h->d_ml_tp;
    Q.gscale = h->d_ml_gs; Q.index = h->d_ml_index;
    // rlearner_grad's form for one step of B samples
    RUnrollParams U;
    std::memset(&U, 0, sizeof(U));
    U.B = B; U.K = K; U.A = A; U.H = h->H;
    U.W = h->rconf.observation_shape[0]; U.P = h->plane; U.obs_feat = h->rin_feat; U.ng = h->rn_ng; U.bn_s = h->bn_s;
    U.plans = h->d_rplan; U.plans_l = h->d_rplan_l; U.ng_l = h->rn_ng_l;
    U.dyn_split = h->rn_dyn_split; U.otab = h->d_rtab;
    U.rd_ep_off = (int)(h->rn_lds_l / 4); U.rd_trunk_nl = 1 + 2 * h->rhp.num_blocks;
    U.rp_nv = 3 + h->rhp.depth_value;
    U.fault = h->d_fault; U.poll_ticks = h->poll_ticks; U.dbg_skip = h->dbg_skip;
    U.ms_wimg = nw; U.ms_flat = fbank_stride(h); U.ms_obs = (size_t)B * (h->ds ? h->rin_feat : h->obs_feat);
    U.ms_k1 = s_k1; U.ms_tp = s_tp; U.ms_hs = (size_t)B * KH * h->H;
    static const bool wide_env = std::getenv("MZ_RN_PRED_WIDE") != nullptr;
    static const bool no_fuse = std::getenv("MZ_RN_NO_FUSE") != nullptr;
    static const bool nb3 = std::getenv("MZ_RN_CHAIN_NB3") != nullptr;
    const bool wide_p = wide_env || (B * KH + U.ng - 1) / U.ng >= h->n_cu;
    const bool fused = h->rd_chain && h->rp_pred && !wide_p && !no_fuse && U.ng_l == 1 && K + 1 < 64 && !h->ds;
    const bool nb1 = (U.P * U.ng_l + 15) / 16 == 1 || !nb3;
    const int gw = A > 16 ? 32 : 16;
    const int nlb = (B * (int)K1 + MZ_THREADS / gw - 1) / (MZ_THREADS / gw);
    double p1 = h->bp1, p2 = h->bp2;
    // chain launches of up to MZ_MULTI_MAX steps (bank half k mod 2), each followed by its steps' unroll
    // launches of up to Ls steps
    const int Lc = std::min(L, std::max(Ls, MZ_MULTI_MAX / Ls * Ls));
    const int R = 2 * MZ_MULTI_MAX / Lc * Lc;       // the per-step scratch ring (ensure_multi)
    for (int k = 0, c0 = 0; c0 < L; ++k, c0 += Lc) {
        const int nc = std::min(Lc, L - c0), half = k & 1, cr = c0 % R;
        ChainParams C;                              // 1. ADAM chain + the nc batches
        std::memset(&C, 0, sizeof(C));
        C.L = nc; C.flat = h->d_flat; C.M = h->d_m; C.V = h->d_v; C.netoff = h->d_netoff;
        C.inv_tile = h->d_inv_tile; C.inv_small = h->d_inv_small;
        C.Wp = h->d_Wp; C.Bp = h->d_Bp; C.smw = h->d_sm_w; C.smb = h->d_sm_bias;
        C.tbank_w = h->d_tbank_w + (size_t)half * MZ_MULTI_MAX * nw;
        C.tbank_b = h->d_tbank_b + (size_t)half * MZ_MULTI_MAX * nb;
        C.tws = nw; C.tbs = nb;
        C.fbank = h->d_fbank + (size_t)half * MZ_MULTI_MAX * fbank_stride(h);
        C.fstride = fbank_stride(h);
        C.theta = theta_dev ? theta_dev + (size_t)c0 * h->nflat : nullptr;
        C.nflat = h->nflat; C.part = h->d_ml_part + (size_t)cr * 3 * MZ_L2_BLOCKS;
        set_caps(C, cap, (int64_t)step0 + c0, nc);
        for (int i = 0; i < nc; ++i) {
            C.bp1[i] = p1; C.bp2[i] = p2; C.eta[i] = eta[c0 + i];
            p1 = p1 * 0.9; p2 = p2 * 0.999;
        }
        RpSampleParams Qc = Q;
        Qc.step = step0 + (uint32_t)c0;
        Qc.obs += cr * s_obs; Qc.actions += cr * s_k1; Qc.tv += cr * s_k1; Qc.tr += cr * s_k1;
        Qc.tpol += cr * s_tp; Qc.gscale += (size_t)cr * B; Qc.index += (size_t)cr * 2 * B;
        C.B = B; C.q = Qc; C.s_obs = s_obs; C.s_k1 = s_k1; C.s_tp = s_tp;
        const int nsb = (nc * B + MZ_THREADS / 64 - 1) / (MZ_THREADS / 64);
        const int nht = chain_helpers(h, C);
        if (nht < 0) return -1;
        hipLaunchKernelGGL(mz_learn_chain, dim3(nht + 3 * MZ_L2_BLOCKS + nsb), dim3(MZ_THREADS), 0, st, C);
        MZ_TRY(h, hipGetLastError());
        for (int j0 = 0; j0 < nc; j0 += Ls) {
            const int n = std::min(Ls, nc - j0), i0 = c0 + j0, ir = i0 % R;
            RpSampleParams Qk = Q;                  // steps step0 + i0 ..
            Qk.step = step0 + (uint32_t)i0;
            Qk.obs += ir * s_obs; Qk.actions += ir * s_k1; Qk.tv += ir * s_k1; Qk.tr += ir * s_k1;
            Qk.tpol += ir * s_tp; Qk.gscale += (size_t)ir * B; Qk.index += (size_t)ir * 2 * B;
            // 2. representation input (Atari: the downsampler with step z's parameters), the unrolls
            U.ms = n;
            U.Wimg = C.tbank_w + (size_t)j0 * nw; U.flat = C.fbank + (size_t)j0 * fbank_stride(h);
            U.obs = Qk.obs; U.actions = Qk.actions;
            if (h->ds) {
                float* y = h->d_ml_dsb + (size_t)ir * B * h->rin_feat;
                if (ds_launch(h, Qk.obs, y, n * B, st, C.fbank + (size_t)j0 * fbank_stride(h), B)) return -1;
                U.obs = y;
            }
            U.pv = h->d_ml_pv + ir * s_k1; U.pp = h->d_ml_pp + ir * s_tp; U.pr = h->d_ml_pr + ir * s_k1;
            U.hs = h->d_ml_hs + (size_t)ir * U.ms_hs; U.ts = h->d_ml_ts + (size_t)ir * U.ms_hs;
            void* args[] = {&U};
            hipEvent_t e0 = nullptr, e1 = nullptr;     // mz_debug_enable flag 4: the unroll launch's duration
            if (h->time_unroll) {
                if (timing_events(h, &e0, &e1)) return -1;
                MZ_TRY(h, hipEventRecord(e0, st));
            }
            if (fused) {
                U.prog = h->d_ml_prog + (size_t)ir * B;
                U.prog_base = (++h->ml_prog_epoch) * 64ull;
                U.n_chain = B; U.fuse_sample = 0; U.n_l2 = 0;
                const int nitems = B * KH * (K > 0 ? 3 : 2);
                MZ_TRY(h, hipLaunchKernel(h->rd_nb == 3 ? (const void*)mz_runroll_fused_r3 : (const void*)mz_runroll_fused_r,
                                          dim3(n * (B + nitems)), dim3(RD_THREADS), args,
                                          std::max(rd_chain_lds(h), rp_pred_lds(h)), st));
            } else {
                if (h->rd_chain)
                    MZ_TRY(h, hipLaunchKernel(h->rd_nb == 3 ? (const void*)mz_runroll_chain_r3
                                                            : (const void*)mz_runroll_chain_r,
                                              dim3((B + U.ng_l - 1) / U.ng_l, 1, n), dim3(RD_THREADS), args,
                                              rd_chain_lds(h), st));
                else
                    MZ_TRY(h, hipLaunchKernel(nb1 ? (const void*)mz_runroll_chain1 : (const void*)mz_runroll_chain,
                                              dim3((B + U.ng_l - 1) / U.ng_l, 1, n), dim3(RN_THREADS), args,
                                              h->rn_lds_l, st));
                if (wide_p)
                    MZ_TRY(h, hipLaunchKernel((const void*)mz_runroll_pred,
                                              dim3((B * KH + U.ng - 1) / U.ng, K > 0 ? 2 : 1, n), dim3(RN_THREADS), args,
                                              runroll_lds(h), st));
                else if (h->rp_pred)
                    MZ_TRY(h, hipLaunchKernel((const void*)mz_runroll_pred_r,
                                              dim3((B * KH + U.ng_l - 1) / U.ng_l, K > 0 ? 2 : 1, n), dim3(RD_THREADS),
                                              args, rp_pred_lds(h), st));
                else
                    MZ_TRY(h, hipLaunchKernel(nb1 ? (const void*)mz_runroll_pred_n1 : (const void*)mz_runroll_pred_n,
                                              dim3((B * KH + U.ng_l - 1) / U.ng_l, K > 0 ? 2 : 1, n), dim3(RN_THREADS),
                                              args, h->rn_lds_l, st));
            }
            if (e1) MZ_TRY(h, hipEventRecord(e1, st));
            // 3. the loss terms and per-step folds (Σθ² from the chain launch)
            LossMultiParams M;
            std::memset(&M, 0, sizeof(M));
            M.B = B; M.K = K; M.A = A; M.v_act = MZ_ACT_IDENTITY; M.r_act = MZ_ACT_IDENTITY; M.nlb = nlb; M.L = n;
            M.s_k1 = s_k1; M.s_tp = s_tp; M.pv = U.pv; M.pp = U.pp; M.pr = U.pr;
            M.tv = Qk.tv; M.tp = Qk.tpol; M.gs = Qk.gscale;
            M.terms = h->d_ml_terms + 2 * ir * s_k1; M.part = h->d_ml_part + (size_t)ir * 3 * MZ_L2_BLOCKS;
            M.counter = h->d_ml_cnt + (size_t)ir * MZ_MULTI_CNT_STRIDE;
            M.out = losses_dev ? losses_dev + 8 * i0 : h->d_ml_out + 8 * ir;
            M.out_last = i0 + n == L ? out_last : nullptr;
            hipLaunchKernelGGL(gw == 32 ? mz_learner_loss_multi32 : mz_learner_loss_multi, dim3(nlb, n), dim3(MZ_THREADS),
                               0, st, M);
            MZ_TRY(h, hipGetLastError());
        }
    }
    const std::string chain = h->rd_chain ? (h->rd_nb == 3 ? "mz_runroll_chain_r3" : "mz_runroll_chain_r")
                                          : nb1 ? "mz_runroll_chain1" : "mz_runroll_chain";
    const std::string pred = wide_p ? "mz_runroll_pred" : h->rp_pred ? "mz_runroll_pred_r"
                                                        : nb1 ? "mz_runroll_pred_n1" : "mz_runroll_pred_n";
    h->last_lvariant = std::string("mz_learn_chain+") + (h->ds ? "mz_downsample_kernel+" : "") +
                       (fused ? (h->rd_nb == 3 ? "mz_runroll_fused_r3" : "mz_runroll_fused_r") : chain + "+" + pred) +
                       "+mz_learner_loss_multi";
    for (int i = 0; i < L; ++i) adam_advance(h);
    h->ml_last_B = B; h->ml_last_L = L; h->ml_last_R = R;
    return 0;
}

// out_last: also (instead of losses[L-1]) the last step's losses there (mz_train_run)
static int learner_multi(mz_handle* h, int32_t B, uint32_t step0, int32_t L, const double* eta, float* losses_dev,
                         float* theta_dev, hipStream_t st, float* out_last = nullptr, const MultiCap* cap = nullptr) {
    MZ_TRY(h, hipSetDevice(h->device));
    if (rmulti_ok(h)) return rlearner_multi(h, B, step0, L, eta, losses_dev, theta_dev, st, out_last, cap);
    int Ls = 0;
    const int ti = multi_ok(h) ? multi_plan(h, B, L, &Ls) : -1;
    if (ti < 0) {
        // the same L steps one launch each (ResNet, the corrected mode, PER, wide nets)
        for (int i = 0; i < L; ++i) {
            float* lo = losses_dev ? losses_dev + 8 * i : (i == L - 1 ? out_last : nullptr);
            if (learner_sampled(h, B, step0 + (uint32_t)i, nullptr, lo, st, true, eta[i])) return -1;
            if (i == L - 1 && out_last && losses_dev)
                MZ_TRY(h, hipMemcpyAsync(out_last, lo, 8 * 4, hipMemcpyDeviceToDevice, st));
            if (theta_dev)
                MZ_TRY(h, hipMemcpyAsync(theta_dev + (size_t)i * h->nflat, h->d_flat, h->nflat * 4,
                                         hipMemcpyDeviceToDevice, st));
            for (int j = 0; j < 2; ++j)
                if (cap && cap->t[j] == (int64_t)step0 + i)
                    MZ_TRY(h, hipMemcpyAsync(cap->dst[j], h->d_flat, h->nflat * 4, hipMemcpyDeviceToDevice, st));
        }
        h->ml_last_L = 0;                           // (no multi-step read-outs: mz_debug_unroll_step refuses)
        return 0;
    }
    RpSampleParams Q;
    mz_batch b;
    if (rs_params(h, B, step0, st, &Q, &b, true)) return -1;   // (the shard; set 0 is not touched)
    if (ensure_batch(h, B) || ensure_multi(h, B, L)) return -1;
    const size_t K1 = (size_t)h->conf.num_unroll_steps + 1, A = (size_t)h->A;
    const size_t s_obs = (size_t)B * h->obs_feat, s_k1 = (size_t)B * K1, s_tp = (size_t)B * K1 * A;
    Q.obs = h->d_ml_obs; Q.actions = h->d_ml_act; Q.tv = h->d_ml_tv; Q.tr = h->d_ml_tr; Q.tpol = h->d_ml_tp;
    Q.gscale = h->d_ml_gs; Q.index = h->d_ml_index;
    static const bool chain_sample = std::getenv("MZ_MULTI_CHAIN_SAMPLE") != nullptr;   // A/B
    SmallUnrollParams U;
    if (small_unroll_params(h, &b, ti, nullptr, &U)) return -1;
    const int T = ti == 2 ? 4 : ti + 1, nU = (B + T - 1) / T;
    static const bool no_xcd = std::getenv("MZ_MULTI_NO_XCD") != nullptr;
    double p1 = h->bp1, p2 = h->bp2;
    // chain launches of up to MZ_MULTI_MAX steps (bank half k mod 2), each followed by its steps' unroll
    // launches of Ls steps (one workgroup per CU)
    const int Lc = std::min(L, std::max(Ls, MZ_MULTI_MAX / Ls * Ls));
    const int R = 2 * MZ_MULTI_MAX / Lc * Lc;       // the per-step scratch ring (ensure_multi)
    for (int k = 0, c0 = 0; c0 < L; ++k, c0 += Lc) {
        const int nc = std::min(Lc, L - c0), half = k & 1, cr = c0 % R;
        // 1. the ADAM chain θ_{t+c0} .. θ_{t+c0+nc} into bank half k mod 2
        ChainParams C;
        std::memset(&C, 0, sizeof(C));
        C.L = nc; C.flat = h->d_flat; C.M = h->d_m; C.V = h->d_v; C.netoff = h->d_netoff;
        C.inv_tile = h->d_inv_tile; C.inv_small = h->d_inv_small;
        C.Wp = h->d_Wp; C.Bp = h->d_Bp; C.smw = h->d_sm_w; C.smb = h->d_sm_bias;
        C.bank_w = h->d_bank_w + (size_t)half * MZ_MULTI_MAX * h->sm_w_n;
        C.bank_b = h->d_bank_b + (size_t)half * MZ_MULTI_MAX * h->sm_b_n;
        C.bws = h->sm_w_n; C.bbs = h->sm_b_n;
        C.theta = theta_dev ? theta_dev + (size_t)c0 * h->nflat : nullptr;
        C.nflat = h->nflat; C.part = h->d_ml_part + (size_t)cr * 3 * MZ_L2_BLOCKS;
        set_caps(C, cap, (int64_t)step0 + c0, nc);
        for (int i = 0; i < nc; ++i) {              // adam_advance's products, step by step
            C.bp1[i] = p1; C.bp2[i] = p2; C.eta[i] = eta[c0 + i];
            p1 = p1 * 0.9; p2 = p2 * 0.999;
        }
        RpSampleParams Qc = Q;                      // this chunk's batches: steps step0 + c0 ..
        Qc.step = step0 + (uint32_t)c0;
        Qc.obs += cr * s_obs; Qc.actions += cr * s_k1; Qc.tv += cr * s_k1; Qc.tr += cr * s_k1;
        Qc.tpol += cr * s_tp; Qc.gscale += (size_t)cr * B; Qc.index += (size_t)cr * 2 * B;
        C.B = B; C.q = Qc; C.s_obs = s_obs; C.s_k1 = s_k1; C.s_tp = s_tp;
        const int nsb = chain_sample ? (nc * B + MZ_THREADS / 64 - 1) / (MZ_THREADS / 64) : 0;
        const int nht = chain_helpers(h, C);
        if (nht < 0) return -1;
        hipLaunchKernelGGL(mz_learn_chain, dim3(nht + 3 * MZ_L2_BLOCKS + nsb), dim3(MZ_THREADS), 0, st, C);
        MZ_TRY(h, hipGetLastError());
        for (int j0 = 0; j0 < nc; j0 += Ls) {
            const int n = std::min(Ls, nc - j0), i0 = c0 + j0, ir = i0 % R;
            RpSampleParams Qk = Q;                  // steps step0 + i0 ..
            Qk.step = step0 + (uint32_t)i0;
            Qk.obs += ir * s_obs; Qk.actions += ir * s_k1; Qk.tv += ir * s_k1; Qk.tr += ir * s_k1;
            Qk.tpol += ir * s_tp; Qk.gscale += (size_t)ir * B; Qk.index += (size_t)ir * 2 * B;
            // 2. the n unrolls (with their get_batch), loss terms and per-step folds
            LearnMultiParams M;
            std::memset(&M, 0, sizeof(M));
            M.L = n; M.nU = nU;
            M.xcd = !no_xcd && n > 1;
            M.bank_w = C.bank_w + (size_t)j0 * h->sm_w_n; M.bank_b = C.bank_b + (size_t)j0 * h->sm_b_n;
            M.bws = h->sm_w_n; M.bbs = h->sm_b_n;
            M.s_obs = s_obs; M.s_k1 = s_k1; M.s_tp = s_tp;
            M.obs = Qk.obs; M.act = Qk.actions; M.tv = Qk.tv; M.tp = Qk.tpol; M.gs = Qk.gscale;
            M.pv = h->d_ml_pv + ir * s_k1; M.pp = h->d_ml_pp + ir * s_tp; M.pr = h->d_ml_pr + ir * s_k1;
            M.terms = h->d_ml_terms + 2 * ir * s_k1;
            M.part = h->d_ml_part + (size_t)ir * 3 * MZ_L2_BLOCKS;
            M.counter = h->d_ml_cnt + (size_t)ir * MZ_MULTI_CNT_STRIDE;
            M.out = losses_dev ? losses_dev + 8 * i0 : h->d_ml_out + 8 * ir;
            M.out_last = i0 + n == L ? out_last : nullptr;
            M.sample = chain_sample ? 0 : 1;
            M.q = Qk;
            const int grid = M.xcd ? 8 * ((n + 7) / 8) * nU : n * nU;
            void* args[] = {&U, &M};
            hipEvent_t e0 = nullptr, e1 = nullptr; // mz_debug_enable flag 4: the unroll launch's duration
            if (h->time_unroll) {
                if (timing_events(h, &e0, &e1)) return -1;
                MZ_TRY(h, hipEventRecord(e0, st));
            }
            const void* kbn[3] = {(const void*)mz_learn_multi1_bn, (const void*)mz_learn_multi2_bn,
                                  (const void*)mz_learn_multi4_bn};
            const void* kpl[3] = {(const void*)mz_learn_multi1, (const void*)mz_learn_multi2,
                                  (const void*)mz_learn_multi4};
            MZ_TRY(h, hipLaunchKernel(h->sm_bn ? kbn[ti] : kpl[ti],
                                      dim3(grid), dim3(SM_THREADS), args, unroll_small_lds(h, ti), st));
            if (e1) MZ_TRY(h, hipEventRecord(e1, st));
        }
    }
    h->last_lvariant = ti == 0 ? "mz_learn_chain+mz_learn_multi1"
                     : ti == 1 ? "mz_learn_chain+mz_learn_multi2" : "mz_learn_chain+mz_learn_multi4";
    for (int i = 0; i < L; ++i) adam_advance(h);
    h->ml_last_B = B; h->ml_last_L = L; h->ml_last_R = R;
    return 0;
}

int mz_learner_train_multi_dev(mz_handle* h, int32_t B, uint32_t step0, int32_t L, const double* eta,
                               float* losses_dev, float* theta_dev, void* stream) {
    if (!h) return -2;
    if (L < 1 || L > MZ_MULTI_LMAX) return fail(h, "L must be in 1 .. 256");
    if (!eta) return fail(h, "eta: one learning rate per step");
    if (B < 1) return fail(h, "batch_size must be >= 1");
    return learner_multi(h, B, step0, L, eta, losses_dev, theta_dev, stream ? (hipStream_t)stream : h->stream);
}

int mz_debug_unroll_step(mz_handle* h, int i, int B, float* values, float* policies, float* rewards) {
    if (!h) return -2;
    if (i < 0 || i >= h->ml_last_L || i < h->ml_last_L - h->ml_last_R || B < 0 || B > h->ml_last_B)
        return fail(h, "no such step / batch in the last mz_learner_train_multi_dev");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    const size_t K1 = (size_t)h->conf.num_unroll_steps + 1, A = (size_t)h->A, s = (size_t)h->ml_last_B * K1;
    const size_t n = (size_t)B * K1;
    const size_t ir = (size_t)(i % h->ml_last_R);   // the ring slot of step i (ensure_multi)
    if (values) MZ_TRY(h, hipMemcpy(values, h->d_ml_pv + ir * s, n * 4, hipMemcpyDeviceToHost));
    if (policies) MZ_TRY(h, hipMemcpy(policies, h->d_ml_pp + ir * s * A, n * A * 4, hipMemcpyDeviceToHost));
    if (rewards) MZ_TRY(h, hipMemcpy(rewards, h->d_ml_pr + ir * s, n * 4, hipMemcpyDeviceToHost));
    return 0;
}

int mz_replay_get_game(mz_handle* h, int32_t i, int32_t* T, uint8_t* obs, int32_t* actions, float* rewards,
                       int32_t* to_play, float* child_visits, float* root_values) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    long long c[3];
    MZ_TRY(h, hipMemcpy(c, h->d_sp_counters, sizeof(c), hipMemcpyDeviceToHost));
    const long long held = std::min<long long>(c[0], h->sp_cap);
    if (i < 0 || i >= held) return fail(h, "game index out of range");
    const long long num = c[0] - held + 1 + i;
    const int slot = (int)((num - 1) % h->sp_cap);
    const size_t base = (size_t)slot * h->sp_T, A = (size_t)h->A;
    const SpHist& r = h->sp_ring;
    int32_t len = 0;
    MZ_TRY(h, hipMemcpy(&len, r.len + slot, 4, hipMemcpyDeviceToHost));
    if (T) *T = len;
    if (obs) MZ_TRY(h, hipMemcpy(obs, r.obs + base * h->sp_osz, (size_t)len * h->sp_osz, hipMemcpyDeviceToHost));
    if (actions) MZ_TRY(h, hipMemcpy(actions, r.act + base, (size_t)len * 4, hipMemcpyDeviceToHost));
    if (rewards) MZ_TRY(h, hipMemcpy(rewards, r.rew + base, (size_t)len * 4, hipMemcpyDeviceToHost));
    if (to_play) MZ_TRY(h, hipMemcpy(to_play, r.tp + base, (size_t)len * 4, hipMemcpyDeviceToHost));
    if (child_visits) MZ_TRY(h, hipMemcpy(child_visits, r.cv + base * A, (size_t)len * A * 4, hipMemcpyDeviceToHost));
    if (root_values) MZ_TRY(h, hipMemcpy(root_values, r.rv + base, (size_t)len * 4, hipMemcpyDeviceToHost));
    return 0;
}

int mz_selfplay_slots(mz_handle* h, int32_t* history_len, uint8_t* board, int32_t* player) {
    if (!h) return -2;
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (h->sp_reset_pending)       // the initial games are keyed by the first move's game_offset
        return fail(h, "the Atari-like env draws its initial games at the first mz_selfplay_move");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    const size_t G = (size_t)h->sp_G;
    if (history_len) MZ_TRY(h, hipMemcpy(history_len, h->sp_hist.len, G * 4, hipMemcpyDeviceToHost));
    if (board) MZ_TRY(h, hipMemcpy(board, h->d_sp_board, G * h->sp_osz, hipMemcpyDeviceToHost));
    if (player) MZ_TRY(h, hipMemcpy(player, h->d_sp_player, G * 4, hipMemcpyDeviceToHost));
    return 0;
}

// ---- actor–learner loop (self_play! ‖ learning!, Q16)
// The actors search with their own weight set; the learner trains the
// engine's weights.  The set is swapped in around each self-play move (the
// search kernels read the images the handle points at).
static void wset_swap(mz_handle* h, mz_handle::WSet& w) {
    std::swap(h->d_flat, w.flat); std::swap(h->d_Wp, w.Wp); std::swap(h->d_Bp, w.Bp);
    std::swap(h->d_sm_w, w.smw); std::swap(h->d_sm_bias, w.smb);
}
// flat -> the set's search images (the repack of the handle's current images)
static int wset_repack(mz_handle* h, mz_handle::WSet& w, hipStream_t st) {
    const int T = 256;
    hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_w_n + T - 1) / T)), dim3(T), 0, st,
                       w.flat, h->d_srcW, w.Wp, h->packed_w_n);
    if (h->packed_b_n)
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->packed_b_n + T - 1) / T)), dim3(T), 0, st,
                           w.flat, h->d_srcB, w.Bp, h->packed_b_n);
    if (h->small_ok) {
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_w_n + T - 1) / T)), dim3(T), 0, st,
                           w.flat, h->d_sm_srcw, w.smw, h->sm_w_n);
        hipLaunchKernelGGL(mz_repack_kernel, dim3((unsigned)((h->sm_b_n + T - 1) / T)), dim3(T), 0, st,
                           w.flat, h->d_sm_srcb, w.smb, h->sm_b_n);
    }
    MZ_TRY(h, hipGetLastError());
    return 0;
}
// ParameterSchedulers 0.2.3 Cos(λ0 = 1e-4, λ1 = 1e-1, period = 10) under
// Stateful, step t >= 1 (Learning.jl:319, 382)
static double cos_schedule(int64_t t) {
    const double l0 = 1e-4, l1 = 1e-1, range = std::fabs(l0 - l1), off = std::min(l0, l1);
    const double a = 6.283185307179586 * (double)(t - 1) / 10.0;
    return range * (1.0 + std::cos(a)) / 2.0 + off;
}

static float temp_fn(int64_t t) { return t < 500000 ? 1.0f : t < 750000 ? 0.5f : 0.25f; }   // SelfPlay.jl:48-56

int mz_train_init(mz_handle* h, int32_t B) { return mz_train_init_at(h, B, 0); }

int mz_train_set_networks_path(mz_handle* h, const char* networks_path) {
    if (!h) return -2;
    h->tr_ckpt_path = networks_path ? networks_path : "";
    return 0;
}

int mz_train_init_at(mz_handle* h, int32_t B, int64_t t0) {
    if (!h) return -2;
    if (t0 < 0) return fail(h, "the starting training step must be >= 0");
    if (h->sp_env < 0) return fail(h, "mz_selfplay_init first");
    if (B < 1) return fail(h, "batch_size must be >= 1");
    if (h->conf.checkpoint_interval < 1) return fail(h, "checkpoint_interval must be >= 1");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    mz_handle::WSet& w = h->tr_actor;
    if (!w.flat) {
        MZ_TRY(h, dalloc(h, &w.flat, h->nflat));
        MZ_TRY(h, dalloc(h, &w.Wp, h->packed_w_n));
        if (h->packed_b_n) MZ_TRY(h, dalloc(h, &w.Bp, h->packed_b_n));
        if (h->small_ok) { MZ_TRY(h, dalloc(h, &w.smw, h->sm_w_n)); MZ_TRY(h, dalloc(h, &w.smb, h->sm_b_n)); }
        MZ_TRY(h, dalloc(h, &h->d_tr_queued, h->nflat));
        MZ_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&h->h_tr_cnt), 4 * sizeof(long long)));
        MZ_TRY(h, hipHostMalloc(reinterpret_cast<void**>(&h->h_tr_pub), 4 * sizeof(long long), hipHostMallocCoherent));
        std::memset(h->h_tr_pub, 0, 4 * sizeof(long long));
        h->tr_pub_seq = 0;
    }
    // actors and the queue start from the learner's current (initial) nets (main.jl:23)
    MZ_TRY(h, hipMemcpyAsync(w.flat, h->d_flat, h->nflat * 4, hipMemcpyDeviceToDevice, h->stream));
    MZ_TRY(h, hipMemcpyAsync(h->d_tr_queued, h->d_flat, h->nflat * 4, hipMemcpyDeviceToDevice, h->stream));
    if (wset_repack(h, w, h->stream)) return -1;
    MZ_TRY(h, hipMemcpyAsync(h->h_tr_cnt, h->d_sp_counters, sizeof(long long), hipMemcpyDeviceToHost, h->stream));
    MZ_TRY(h, hipStreamSynchronize(h->stream));
    // games already in progress keep visit_softmax_temperature_fn(t0) to their end
    std::vector<float> tg((size_t)h->sp_G, temp_fn(t0));
    MZ_TRY(h, hipMemcpy(h->d_sp_tgame, tg.data(), tg.size() * 4, hipMemcpyHostToDevice));
    h->tr_B = B; h->tr_t = t0; h->tr_refresh = 0;
    h->tr_games = h->h_tr_cnt[0];
    return 0;
}

// the move's hand-back to the host: the finished-game count and the fault word, then a sequence
// number, stored into coherent pinned host memory at system scope; the host spins on the sequence
// number instead of two copy launches and a stream synchronisation (measured in the trace: 30-60 us
// from the copies' end to the next launch)
extern "C" __global__ void mz_tr_publish(const long long* counters, const unsigned* fault, long long* host,
                                         long long seq) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(host + 0, counters[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host + 1, fault ? (long long)*fault : 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// wait for publish `seq` (bounded: after 60 s the stream is synchronised, which reports a launch error)
static int tr_wait_publish(mz_handle* h, long long seq, hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned n = 0; __atomic_load_n(h->h_tr_pub + 2, __ATOMIC_ACQUIRE) != seq; ++n) {
        if ((n & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
            MZ_TRY(h, hipStreamSynchronize(st));
            if (__atomic_load_n(h->h_tr_pub + 2, __ATOMIC_ACQUIRE) == seq) break;
            return fail(h, "mz_train: the move's publish never arrived");
        }
        __builtin_ia32_pause();
    }
    return 0;
}

// 1. one self-play move with the actors' nets (SelfPlay.jl:343-380); temperature
//    visit_softmax_temperature_fn(t) (:48-56, 396-397) for the games that start on
//    this move (a game in progress keeps its own).  *nfin = the games save_game
//    stored (slot order, inside the move).  The fault word rides along with the
//    counter copy: one stream wait per move, no second blocking copy.
static int train_move(mz_handle* h, uint32_t move, uint32_t game_offset, int64_t* nfin, hipStream_t st) {
    const float temp = temp_fn(h->tr_t);
    wset_swap(h, h->tr_actor);
    h->sp_latch = true;
    const int rc = mz_selfplay_move(h, move, game_offset, temp, st);
    h->sp_latch = false;
    wset_swap(h, h->tr_actor);
    if (rc) return rc;
    static const bool copy_sync = std::getenv("MZ_TRAIN_SYNC") != nullptr;   // A/B: round 6's copies + sync
    if (copy_sync) {
        MZ_TRY(h, hipMemcpyAsync(h->h_tr_cnt, h->d_sp_counters, sizeof(long long), hipMemcpyDeviceToHost, st));
        h->h_tr_cnt[1] = 0;
        if (h->d_fault) MZ_TRY(h, hipMemcpyAsync(h->h_tr_cnt + 1, h->d_fault, 4, hipMemcpyDeviceToHost, st));
        MZ_TRY(h, hipStreamSynchronize(st));
    } else {
        const long long seq = ++h->tr_pub_seq;
        hipLaunchKernelGGL(mz_tr_publish, dim3(1), dim3(64), 0, st, (const long long*)h->d_sp_counters,
                           (const unsigned*)h->d_fault, h->h_tr_pub, seq);
        MZ_TRY(h, hipGetLastError());
        if (tr_wait_publish(h, seq, st)) return -1;
        h->h_tr_cnt[0] = h->h_tr_pub[0];
        h->h_tr_cnt[1] = h->h_tr_pub[1];
    }
    if (h->h_tr_cnt[1] && check_fault(h)) return -1;
    *nfin = h->h_tr_cnt[0] - h->tr_games;
    h->tr_games = h->h_tr_cnt[0];
    return 0;
}

// the actors take the queued nets, the learner's nets are queued (SelfPlay.jl:399-401 /
// Learning.jl:416-418: one checkpoint behind); past round(0.9 training_steps) the nets
// go to disk (Learning.jl:427-432, round half to even as Julia's round)
static int train_refresh(mz_handle* h, int64_t t, hipStream_t st) {
    MZ_TRY(h, hipMemcpyAsync(h->tr_actor.flat, h->d_tr_queued, h->nflat * 4, hipMemcpyDeviceToDevice, st));
    if (wset_repack(h, h->tr_actor, st)) return -1;
    MZ_TRY(h, hipMemcpyAsync(h->d_tr_queued, h->d_flat, h->nflat * 4, hipMemcpyDeviceToDevice, st));
    ++h->tr_refresh;
    if (!h->tr_ckpt_path.empty() && (double)t > std::nearbyint(0.9 * (double)h->conf.training_steps)) {
        MZ_TRY(h, hipStreamSynchronize(st));
        const std::string path = h->tr_ckpt_path + "/" + std::to_string(t) + ".safetensors";
        if (mz_checkpoint_save(h, path.c_str(), t)) return -1;
    }
    return 0;
}

// 2. `nreq` learner steps while t <= training_steps (Learning.jl:327), get_batch keyed by
//    the step number, eta = Cos(step); every checkpoint_interval steps (t % ci == 0, t > 1)
//    an actor refresh.  Round 6: the steps of one call run as ONE mz_learner_train_multi_dev
//    chunk across the refresh points (up to 256 steps per call; MZ_TRAIN_L caps it): nothing
//    reads the actors' or the queued nets between two learner steps of one move, so only
//    the sets after the last refresh matter — θ of the last refresh step is queued, θ of the
//    one before it (or, with one refresh, the previously queued nets) goes to the actors, and
//    the chain launch that computes those θ copies them out (MultiCap).  With periodic
//    checkpoint files (networks_path) or MZ_TRAIN_PER_REFRESH=1 the chunks end at every
//    refresh step as in round 5 (the checkpoint writes the learner's nets of that step).
static int train_learn(mz_handle* h, int64_t nreq, float* losses_dev, hipStream_t st, int64_t* done) {
    static const int chunk_env = std::getenv("MZ_TRAIN_L") ? std::atoi(std::getenv("MZ_TRAIN_L")) : 0;
    static const bool per_refresh_env = std::getenv("MZ_TRAIN_PER_REFRESH") != nullptr;
    const int chunk_max = std::max(1, std::min(MZ_MULTI_LMAX, chunk_env > 0 ? chunk_env : MZ_MULTI_LMAX));
    const bool per_refresh = per_refresh_env || !h->tr_ckpt_path.empty();
    const int64_t ci = h->conf.checkpoint_interval;
    auto is_refresh = [&](int64_t t) { return t % ci == 0 && t > 1; };
    const int64_t n_all = std::max<int64_t>(0, std::min<int64_t>(nreq, (int64_t)h->conf.training_steps + 1 - h->tr_t));
    *done = 0;
    if (n_all == 0) return 0;
    // the actors' set: θ of the next-to-last refresh step, its search images written by the chain launch
    // that computes it (else repacked after the call)
    bool imaged = false;
    static const bool no_cap_img = std::getenv("MZ_TRAIN_REPACK") != nullptr;   // A/B
    MultiCap cap{{-1, -1}, {h->tr_actor.flat, h->d_tr_queued}, no_cap_img ? nullptr : &h->tr_actor, &imaged};
    int64_t nref = 0;
    if (!per_refresh) {
        // the refresh steps in (t, t + n]: the last two
        const int64_t t_lo = h->tr_t, t_hi = h->tr_t + n_all;
        for (int64_t r = t_hi / ci * ci; r > t_lo && nref < 2; r -= ci)
            if (is_refresh(r)) { cap.t[1 - nref] = r; ++nref; }
        const int64_t first = (t_lo / ci + 1) * ci;   // the total count
        nref = 0;
        for (int64_t r = first; r <= t_hi; r += ci) nref += is_refresh(r) ? 1 : 0;
        if (nref == 1) {               // the actors take the nets queued before this call
            MZ_TRY(h, hipMemcpyAsync(h->tr_actor.flat, h->d_tr_queued, h->nflat * 4, hipMemcpyDeviceToDevice, st));
            cap.t[0] = -1;
        }
    }
    double eta[MZ_MULTI_LMAX];
    for (int64_t k = 0; k < n_all;) {
        const int64_t t0 = h->tr_t + 1;
        int64_t n = std::min<int64_t>(n_all - k, chunk_max);
        if (per_refresh) {                                 // the chunk ends at the next refresh step
            int64_t tb = (t0 + ci - 1) / ci * ci;
            if (tb <= 1) tb += ci;
            n = std::min<int64_t>(n, tb - t0 + 1);
        }
        const int64_t t = t0 + n - 1;
        if (n == 1) {
            if (mz_learner_train_dev(h, h->tr_B, (uint32_t)t, cos_schedule(t), losses_dev, st)) return -1;
            for (int j = 0; j < 2; ++j)
                if (cap.t[j] == t)
                    MZ_TRY(h, hipMemcpyAsync(cap.dst[j], h->d_flat, h->nflat * 4, hipMemcpyDeviceToDevice, st));
        } else {
            for (int64_t i = 0; i < n; ++i) eta[i] = cos_schedule(t0 + i);
            if (learner_multi(h, h->tr_B, (uint32_t)t0, (int32_t)n, eta, nullptr, nullptr, st, losses_dev,
                              per_refresh ? nullptr : &cap))
                return -1;
        }
        h->tr_t = t;
        *done += n;
        k += n;
        if (per_refresh && is_refresh(t) && train_refresh(h, t, st)) return -1;
    }
    if (!per_refresh && nref > 0) {
        if (!(nref >= 2 && imaged) && wset_repack(h, h->tr_actor, st)) return -1;
        h->tr_refresh += nref;
    }
    return 0;
}

// a count summed over the ranks of the handle's RCCL communicator (exact below 2^24)
static int dp_sum_count(mz_handle* h, int64_t* v, hipStream_t st) {
    if (!h->d_dp_cnt) MZ_TRY(h, dalloc(h, &h->d_dp_cnt, 1));
    float f = (float)*v;
    MZ_TRY(h, hipMemcpyAsync(h->d_dp_cnt, &f, 4, hipMemcpyHostToDevice, st));
    const int rc = rccl().allreduce(h->d_dp_cnt, h->d_dp_cnt, 1, 7, 0, h->dp_comm, st);   // ncclFloat32, ncclSum
    if (rc != 0) return fail(h, std::string("ncclAllReduce: ") + (rccl().err ? rccl().err(rc) : "error"));
    MZ_TRY(h, hipMemcpyAsync(&f, h->d_dp_cnt, 4, hipMemcpyDeviceToHost, st));
    MZ_TRY(h, hipStreamSynchronize(st));
    *v = (int64_t)f;
    return 0;
}

int mz_train_move(mz_handle* h, uint32_t move, uint32_t game_offset, int64_t* nfin, void* stream) {
    if (!h) return -2;
    if (!h->tr_B) return fail(h, "mz_train_init first");
    MZ_TRY(h, hipSetDevice(h->device));
    int64_t n = 0;
    if (train_move(h, move, game_offset, &n, stream ? (hipStream_t)stream : h->stream)) return -1;
    if (nfin) *nfin = n;
    return 0;
}

int mz_train_learn(mz_handle* h, int64_t steps, float* losses_dev, int64_t* state_out, void* stream) {
    if (!h) return -2;
    if (!h->tr_B) return fail(h, "mz_train_init first");
    if (steps < 0) return fail(h, "steps must be >= 0");
    MZ_TRY(h, hipSetDevice(h->device));
    int64_t done = 0;
    if (train_learn(h, steps, losses_dev, stream ? (hipStream_t)stream : h->stream, &done)) return -1;
    if (state_out) {
        state_out[0] = h->tr_t; state_out[1] = h->tr_games; state_out[2] = h->tr_refresh; state_out[3] = done;
    }
    return 0;
}

int mz_train_run(mz_handle* h, int32_t moves, uint32_t move0, uint32_t game_offset, int64_t* state_out,
                 float* losses_dev, void* stream) {
    if (!h) return -2;
    if (!h->tr_B) return fail(h, "mz_train_init first");
    if (moves < 0) return fail(h, "moves must be >= 0");
    MZ_TRY(h, hipSetDevice(h->device));
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    int64_t steps = 0;
    for (int32_t mv = 0; mv < moves; ++mv) {
        int64_t nfin = 0, done = 0;
        if (train_move(h, move0 + (uint32_t)mv, game_offset, &nfin, st)) return -1;
        // data parallel (mz_dp_init): every rank takes the learner steps of the games all
        // ranks finished, so the replicas stay identical
        if (h->dp_comm && h->dp_world > 1 && dp_sum_count(h, &nfin, st)) return -1;
        if (train_learn(h, nfin, losses_dev, st, &done)) return -1;
        steps += done;
    }
    if (state_out) {
        state_out[0] = h->tr_t; state_out[1] = h->tr_games; state_out[2] = h->tr_refresh; state_out[3] = steps;
    }
    return 0;
}

int mz_train_weights_get(mz_handle* h, int which, int net, float* flat, size_t n) {
    if (!h) return -2;
    if (which == MZ_TRAIN_LEARNER) return mz_weights_get(h, net, flat, n);
    if (!h->tr_B) return fail(h, "mz_train_init first");
    if (which != MZ_TRAIN_ACTOR && which != MZ_TRAIN_QUEUED) return fail(h, "which: learner, actor or queued");
    if (net < 0 || net > 2) return fail(h, "bad net id");
    if (n != h->nparams[net]) return fail(h, "wrong parameter count");
    MZ_TRY(h, hipSetDevice(h->device));
    MZ_SYNC(h);
    const float* src = which == MZ_TRAIN_ACTOR ? h->tr_actor.flat : h->d_tr_queued;
    MZ_TRY(h, hipMemcpy(flat, src + h->flat_off[net], n * 4, hipMemcpyDeviceToHost));
    return 0;
}

int mz_sync(mz_handle* h) {
    if (!h) return -2;
    MZ_TRY(h, hipSetDevice(h->device));
    // every stream `_dev` work may have gone to (the device, or the narrowed pair of
    // mz_set_sync_stream), so a fault of work queued on a caller stream is reported here
    MZ_SYNC(h);
    return 0;
}

}  // extern "C"
