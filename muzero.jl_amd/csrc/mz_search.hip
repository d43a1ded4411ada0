// mz_search.hip — batched MCTS (run_mcts + select_action + store_search_stats!)
// as ONE persistent kernel launch per move (reference: src/SelfPlay.jl:230-306).
//
// Workgroup = 256 threads = a tile of 16 games.  The kernel runs the root
// inference (representation + prediction, :234,:239), the root expansion and
// Dirichlet noise (:245-249), then loops over the S simulations (:254-283)
// with no grid-wide synchronisation — games are independent:
//
//   select   (:261-268)  16 lanes per game, one child slot per lane (tree in LDS)
//   gather   (:271-273)  parent hidden state -> prediction input; h *= 2 in place
//                        in HBM (Q1) -> dynamics input with the a/|A| plane
//   nets     (:271,:275) prediction ‖ dynamics as one 8-stage f32-MFMA plan
//   expand   (:280)      double softmax (Q3) over the root's legal set (Q4)
//   backup   (:281)      Q7 along the recorded path, per-game min-max stats
//
// The tree (mz_tree_device.h layout, 12 B per edge) lives in LDS when
// 16 games of it fit beside the activations (TicTacToe: S <= 50), otherwise
// in HBM (the <false> instantiation).  Hidden states are in HBM [G][S+1][H].
#include "mz_mlp_device.h"
#include "mz_tree_device.h"

// Diagnostic phase stamps (separate -DMZ_STAMPS build; never in the product
// library): wave 0 lane 0 accumulates s_memtime deltas per phase.
#ifdef MZ_STAMPS
#define MZ_STAMP(i)                                                              \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                \
            st_acc[i] += t_ - st_last; st_last = t_;                             \
        }                                                                        \
    } while (0)
#else
#define MZ_STAMP(i) do {} while (0)
#endif


template <bool LDS_TREE, bool RES>
__device__ __forceinline__ void search_body(const SearchParams& P) {
#ifdef MZ_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* act = smem;
    int* si = reinterpret_cast<int*>(smem + P.lay.total);
    uint32_t* sg_legal = reinterpret_cast<uint32_t*>(si);
    int* sg_root_tp = si + 16;
    int* sg_rootN = si + 32;
    float* sg_rootW = reinterpret_cast<float*>(si + 48);
    float* sg_mmin = reinterpret_cast<float*>(si + 64);
    float* sg_mmax = reinterpret_cast<float*>(si + 80);
    int* sg_leaf_e = si + 96;
    int* sg_leaf_a = si + 112;
    int* sg_vtp = si + 128;
    int* sg_depth = si + 144;
    const int PS = 2 * (P.S + 2);
    float* sg_stage = reinterpret_cast<float*>(si + 160);      // [16][16] seqsum staging
    int* sg_path = si + 416;                                   // [16][2(S+2)]
    char* lds_tree = reinterpret_cast<char*>(si + 416 + 16 * PS);

    const int tid = threadIdx.x, lane = tid & 63;
    const int g = tid >> 4, a = tid & 15;
    const int A = P.A, S = P.S, H = P.H;
    const int E = (S + 1) * A, NN = S + 1;
    const int tile0 = blockIdx.x * MZ_TILE;
    const int gg = tile0 + g;
    const bool active = gg < P.G;
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    int* path = sg_path + g * PS;
    TreeView gtree = tree_view(P.tree + (size_t)(active ? gg : 0) * P.tree_game_bytes, E, NN);
    TreeView tree = LDS_TREE ? tree_view(lds_tree + (size_t)g * P.tree_game_bytes, E, NN) : gtree;

    for (int i = tid; i < P.lay.total; i += blockDim.x) act[i] = 0.0f;
    __syncthreads();

    // ---- root inputs: stacked observation (W,H,Cs,G) -> x_rep[k][g]
    for (int i = tid; i < MZ_TILE * P.obs_feat; i += blockDim.x) {
        const int gl = i / P.obs_feat, k = i - gl * P.obs_feat;
        const int ggl = tile0 + gl;
        act[P.lay.x_rep + k * 16 + gl] = ggl < P.G ? P.obs[(size_t)ggl * P.obs_feat + k] : 0.0f;
    }
    if (a == 0) {
        uint32_t m = 0;
        if (active)
            for (int b = 0; b < A; ++b) if (P.legal[(size_t)gg * A + b]) m |= 1u << b;
        sg_legal[g] = m;
        sg_root_tp[g] = active ? P.to_play[gg] : 1;
        sg_rootN[g] = 0; sg_rootW[g] = 0.0f;
        sg_mmin[g] = INFINITY; sg_mmax[g] = -INFINITY;          // MinMaxStats(Inf, -Inf), :251
    }
    __syncthreads();

    // prediction ‖ dynamics weights stay in registers for all S simulations
    float wr[16 * MZ_RES_TASKS];
    if (RES) res_load(P.plan_sim_res, wr, P.Wp);

    // ---- representation (:234) -> h_out, prediction(h) (:239) -> v_out, p_out
    run_plan(P.plan_root, P.Wp, P.Bp, act);

    for (int i = tid; i < MZ_TILE * H; i += blockDim.x) {
        const int gl = i / H, k = i - gl * H;
        const int ggl = tile0 + gl;
        if (ggl < P.G) P.hid[(size_t)ggl * (S + 1) * H + k] = act[P.lay.h_out + k * 16 + gl];
    }
    const uint32_t legal = sg_legal[g];
    {   // expand_node!(root, legal, to_play, 0, policy, h) (:245)
        const float prior = double_softmax_prior(a < A ? act[P.lay.p_out + a * 16 + g] : 0.0f, a, A, legal,
                                                 sg_stage + 16 * g);
        if (active) {
            init_edges(tree, 0, a, A, prior);
            if (a == 0) { tree.nr[0] = 0.0f; tree.ntp[0] = (int8_t)sg_root_tp[g]; }
        }
    }
    __syncthreads();
    if (P.exploration && active) {                           // add_exploration_noise! (:102-109)
        const float nz = root_noise_lane(legal, a, A, P.seed, gid, P.rng_step, P.dirichlet_alpha, sg_stage + 16 * g);
        if (a < A && ((legal >> a) & 1u)) tree.p(a) = tree.p(a) * (1.0f - P.exploration_eps) + nz * P.exploration_eps;
    }
    __syncthreads();
    MZ_STAMP(0);

    // ---------------------------------------------------------------- simulations
    for (int s = 0; s < S; ++s) {
        // ---- select (:256-268)
        if (active) {
            const SelectOut so = select_path<false>(tree, path, sg_rootN[g], sg_root_tp[g], legal, sg_mmin[g], sg_mmax[g],
                                             a, lane, A, P.players, P.discount, nullptr, P.pbc_tab, P.sqrt_tab, P.seed,
                                             gid, P.rng_step, s);
            if (a == 0) { sg_leaf_e[g] = so.leaf_e; sg_leaf_a[g] = so.leaf_a; sg_vtp[g] = so.vtp; sg_depth[g] = so.depth; }
        }
        __syncthreads();
        MZ_STAMP(1);

        // ---- gather: prediction(parent.h) input; make_state_action doubles h in place (Q1)
        for (int i = tid; i < MZ_TILE * H; i += blockDim.x) {
            const int gl = i / H, k = i - gl * H;
            const int ggl = tile0 + gl;
            if (ggl < P.G) {
                float* hp = P.hid + ((size_t)ggl * (S + 1) + sg_leaf_e[gl]) * H + k;
                const float hv = *hp;
                const float h2 = hv * 2.0f;
                *hp = h2;
                act[P.lay.x_pred + k * 16 + gl] = hv;
                act[P.lay.x_dyn + k * 16 + gl] = h2;
            }
        }
        for (int i = tid; i < MZ_TILE * P.plane; i += blockDim.x) {
            const int gl = i / P.plane, k = i - gl * P.plane;
            if (tile0 + gl < P.G) act[P.lay.x_dyn + (H + k) * 16 + gl] = P.aval_tab[sg_leaf_a[gl]];
        }
        __syncthreads();
        MZ_STAMP(2);

        // ---- prediction(parent.h) ‖ dynamics(2h ⊕ a/|A|)
        if (RES) res_run(P.plan_sim_res, wr, P.Bp, act);
        else run_plan(P.plan_sim, P.Wp, P.Bp, act);
        MZ_STAMP(3);

        // ---- expand the leaf as slot s+1 (:280)
        const int e_new = s + 1;
        {
            const float prior = double_softmax_prior(a < A ? act[P.lay.p_out + a * 16 + g] : 0.0f, a, A, legal,
                                                     sg_stage + 16 * g);
            if (active) init_edges(tree, e_new, a, A, prior);
        }
        for (int i = tid; i < MZ_TILE * H; i += blockDim.x) {
            const int gl = i / H, k = i - gl * H;
            const int ggl = tile0 + gl;
            if (ggl < P.G) P.hid[((size_t)ggl * (S + 1) + e_new) * H + k] = act[P.lay.h_out + k * 16 + gl];
        }
        MZ_STAMP(4);
        // ---- backpropagate! (:190-217)
        if (active) {
            const int tl = sg_vtp[g];
            const int depth = sg_depth[g];
            if (a == 0) {
                const int li = sg_leaf_e[g] * A + sg_leaf_a[g];
                tree.nc(li) = (tree.nc(li) & 0xffffu) | ((uint32_t)(e_new + 1) << 16);
                tree.nr[e_new] = mz_post_act(P.lay.r_act, act[P.lay.r_out + g]);
                tree.ntp[e_new] = (int8_t)tl;
                path[2 * depth + 1] = e_new;
            }
            __builtin_amdgcn_wave_barrier();
            int rN = sg_rootN[g];
            float rW = sg_rootW[g], mmin = sg_mmin[g], mmax = sg_mmax[g];
            backup_path(tree, path, depth, mz_post_act(P.lay.v_act, act[P.lay.v_out + g]), tl, A, P.players, P.discount, rN, rW,
                        sg_root_tp[g], mmin, mmax, a);
            if (a == 0) { sg_rootN[g] = rN; sg_rootW[g] = rW; sg_mmin[g] = mmin; sg_mmax[g] = mmax; }
        }
        __syncthreads();
        MZ_STAMP(5);
    }

    // ---- store_search_stats! (:115-122) + select_action (:293-306)
    if (active) {
        const bool lg = a < A && ((legal >> a) & 1u);
        const int Nc = lg ? (int)(tree.nc(a) & 0xffffu) : 0;
        const int sum = g16_isum(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
        const int act = select_action_dev<16>(Nc, legal, A, P.temp_g ? P.temp_g[gg] : P.temperature, r);
        if (a == 0) {
            const int rN = sg_rootN[g];
            P.root_value[gg] = rN == 0 ? 0.0f : sg_rootW[g] / (float)rN;
            P.action_out[gg] = act + 1;
        }
        if (LDS_TREE && P.dump_tree) dump_tree(tree, gtree, E, NN, a);
    }
#ifdef MZ_STAMPS
    MZ_STAMP(6);
    if (threadIdx.x == 0 && P.stamps)
        for (int i = 0; i < 8; ++i) P.stamps[blockIdx.x * 8 + i] = st_acc[i];
#endif
}

extern "C" __global__ __launch_bounds__(MZ_THREADS, 1) void mz_search_kernel_lds_res(SearchParams P) {
    search_body<true, true>(P);
}
extern "C" __global__ __launch_bounds__(MZ_THREADS, 1) void mz_search_kernel_hbm_res(SearchParams P) {
    search_body<false, true>(P);
}
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_search_kernel_lds(SearchParams P) {
    search_body<true, false>(P);
}
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_search_kernel_hbm(SearchParams P) {
    search_body<false, false>(P);
}
