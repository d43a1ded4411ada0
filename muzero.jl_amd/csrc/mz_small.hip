// mz_small.hip — batched MCTS for SMALL batches (G <= 4 x #CUs): one 256-
// thread workgroup per T in {1, 2, 4} games, so G = 512 spreads over all 256
// CUs of an MI355X instead of the 32 tiles of the 16-game MFMA kernel
// (mz_search.hip), and each simulation waits for the deepest of T games only.
//
// Networks with v_mfma_f32_4x4x1_16b_f32 (16 blocks x 4 rows = one 64-row
// Dense layer, 4 columns = up to 4 games, K = 1 per instruction: a chain of
// them is a k-ordered fmaf chain, bit for bit — tools/mfma4x4_probe.hip).
// Wave q of the workgroup runs k-quarter q of the canonical dot order
// (mz_dot): kq steps over k in [q*kq, (q+1)*kq), weights resident as the MFMA
// A operand for the whole search.  Every wave serves TWO layers ("slots") per
// stage; a layer narrower than 64 rows uses only some 4-row blocks, and a slot
// may hold several such layers (block b reads its own input: the B operand of
// lane 4b+g is game g of that block's input).  The four quarter partials meet
// in LDS and one combine pass forms ((p0+p1)+(p2+p3)) + b and the activation.
// Tree (mz_tree_device.h) and hidden states live in LDS; the host builds the
// stage schedule (mz_engine.hip, build_small_schedule).
#include "mz_mlp_device.h"
#include "mz_tree_device.h"

#include "mz_small_params.h"

#ifdef MZ_STAMPS
#define SM_STAMP(i)                                                              \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                \
            st_acc[i] += t_ - st_last; st_last = t_;                             \
        }                                                                        \
    } while (0)
#else
#define SM_STAMP(i) do {} while (0)
#endif

// One stage: both slots' quarter chains, partials to LDS, combine.
template <int T>
__device__ __forceinline__ void sm_stage(const float (&wa)[16], const float (&wb)[16], const int* rec,
                                         float* lds, float* part) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ka = rec[0], kb = rec[1];
    const int xa = rec[2 + lane], xb = rec[2 + 64 + lane];
    sm_f32x4 da = {0.f, 0.f, 0.f, 0.f}, db = da;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (j < ka) {
            const float va = xa >= 0 ? lds[xa + (q * ka + j) * T] : 0.0f;
            da = __builtin_amdgcn_mfma_f32_4x4x1f32(wa[j], va, da, 0, 0, 0);
        }
        if (j < kb) {
            const float vb = xb >= 0 ? lds[xb + (q * kb + j) * T] : 0.0f;
            db = __builtin_amdgcn_mfma_f32_4x4x1f32(wb[j], vb, db, 0, 0, 0);
        }
    }
    // partials: part[slot][q][lane][4]
    *reinterpret_cast<sm_f32x4*>(part + ((0 * 4 + q) * 64 + lane) * 4) = da;
    *reinterpret_cast<sm_f32x4*>(part + ((1 * 4 + q) * 64 + lane) * 4) = db;
    __syncthreads();
    // combine: output (slot, row r, game g) <- D lane 4*(r/4) + g, reg r%4
    const int* obp = rec + 2 + 128;
    for (int i = tid; i < SM_SLOTS * 64 * T; i += SM_THREADS) {
        const int sl = i / (64 * T), rem = i - sl * 64 * T;
        const int r = rem / T, gm = rem - r * T;
        const int o = obp[sl * 64 + r];
        if (o >= 0) {
            const int src = (4 * (r >> 2) + gm) * 4 + (r & 3);
            const float p0 = part[(sl * 4 + 0) * 256 + src], p1 = part[(sl * 4 + 1) * 256 + src];
            const float p2 = part[(sl * 4 + 2) * 256 + src], p3 = part[(sl * 4 + 3) * 256 + src];
            const float d = ((p0 + p1) + (p2 + p3)) + __int_as_float(obp[128 + sl * 64 + r]);
            lds[o + gm] = obp[256 + sl * 64 + r] ? mz_relu(d) : d;
        }
    }
    __syncthreads();
}

template <int T, int NMAX, int K = 0>
__device__ __forceinline__ void sm_run(int n, const float (&wr)[NMAX][SM_SLOTS][16], const int* rec, float* lds,
                                       float* part) {
    if constexpr (K < NMAX) {
        if (K < n) {
            sm_stage<T>(wr[K][0], wr[K][1], rec + K * SM_REC_INTS, lds, part);
            sm_run<T, NMAX, K + 1>(n, wr, rec, lds, part);
        }
    }
}

template <int NMAX>
__device__ __forceinline__ void sm_load(int n, const float* W, float (&wr)[NMAX][SM_SLOTS][16]) {
    const int tid = threadIdx.x;          // = q * 64 + lane
#pragma unroll
    for (int k = 0; k < NMAX; ++k)
#pragma unroll
        for (int sl = 0; sl < SM_SLOTS; ++sl) {
            if (k < n) {
                const float4* src =
                    reinterpret_cast<const float4*>(W + (((size_t)k * SM_SLOTS + sl) * SM_THREADS + tid) * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 v = src[i];
                    wr[k][sl][4 * i] = v.x; wr[k][sl][4 * i + 1] = v.y;
                    wr[k][sl][4 * i + 2] = v.z; wr[k][sl][4 * i + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) wr[k][sl][i] = 0.0f;
            }
        }
}

// once-per-move helpers kept out of line
__device__ __noinline__ void sm_root_noise(float* p, uint32_t legal, int A, uint64_t seed, uint32_t gid,
                                           uint32_t step, float alpha, float eps) {
    const int n = __builtin_popcount(legal);
    float noise[MZ_MAX_ACTIONS];
    mz_dirichlet(seed, gid, step, n, alpha, noise);
    const float one_m = 1.0f - eps;
    int i = 0;
    for (int b = 0; b < A; ++b) if ((legal >> b) & 1u) {
        p[b] = p[b] * one_m + noise[i] * eps;
        ++i;
    }
}

__device__ __noinline__ int sm_select_action(const int* cnt, uint32_t legal, int A, float temperature, uint32_t r) {
    return select_action_dev(cnt, legal, A, temperature, r);
}

__device__ __forceinline__ TreeView sm_tree_at(char* base, int E, int NN) {
    TreeView t;
    t.nc = reinterpret_cast<uint32_t*>(base);
    t.w = reinterpret_cast<float*>(base + 4 * (size_t)E);
    t.p = reinterpret_cast<float*>(base + 8 * (size_t)E);
    t.nr = reinterpret_cast<float*>(base + 12 * (size_t)E);
    t.ntp = reinterpret_cast<int8_t*>(base + 12 * (size_t)E + 4 * (size_t)NN);
    return t;
}

template <int T>
__device__ __forceinline__ void small_body(const SmallParams& P) {
#ifdef MZ_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int A = P.A, S = P.S, H = P.H;
    const int E = (S + 1) * A, NN = S + 1;
    const int PS = 2 * (S + 2);
    const int nrec = P.n_sim + P.n_root;
    float* act = smem;                                           // act_total floats (multiple of 4)
    float* part = act + P.act_total;                             // [2][4][64][4]
    int* rec = reinterpret_cast<int*>(part + 2048);              // [nrec][SM_REC_INTS]
    float* hid = reinterpret_cast<float*>(rec + (nrec * SM_REC_INTS + 3) / 4 * 4);   // [T][S+1][H]
    int* si = reinterpret_cast<int*>(hid + ((size_t)T * NN * H + 3) / 4 * 4);
    uint32_t* sg_legal = reinterpret_cast<uint32_t*>(si);       // 16-entry blocks
    int* sg_root_tp = si + 16;
    int* sg_rootN = si + 32;
    float* sg_rootW = reinterpret_cast<float*>(si + 48);
    float* sg_mmin = reinterpret_cast<float*>(si + 64);
    float* sg_mmax = reinterpret_cast<float*>(si + 80);
    int* sg_leaf_e = si + 96;
    int* sg_leaf_a = si + 112;
    int* sg_vtp = si + 128;
    int* sg_depth = si + 144;
    float* sg_stage = reinterpret_cast<float*>(si + 160);       // [4][16]
    int* sg_path = si + 224;                                      // [T][2(S+2)]
    char* lds_tree = reinterpret_cast<char*>(si + 224 + (T * PS + 3) / 4 * 4);

    const int tid = threadIdx.x;
    const int g = tid >> 4, a = tid & 15, lane = tid & 63;
    const int tile0 = blockIdx.x * T;
    const bool tree_thread = tid < 16 * T;
    const int gg = tile0 + g;
    const bool active = tree_thread && gg < P.G;
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    int* path = sg_path + (tree_thread ? g : 0) * PS;
    TreeView tree = sm_tree_at(lds_tree + (size_t)(tree_thread ? g : 0) * P.tree_game_bytes, E, NN);
    const int* rec_sim = rec;
    const int* rec_root = rec + P.n_sim * SM_REC_INTS;

    for (int i = tid; i < P.act_total; i += SM_THREADS) act[i] = 0.0f;
    for (int i = tid; i < nrec * SM_REC_INTS; i += SM_THREADS) rec[i] = P.rec[i];
    __syncthreads();
    for (int i = tid; i < nrec * 128; i += SM_THREADS)
        rec[(i >> 7) * SM_REC_INTS + 258 + (i & 127)] = __float_as_int(P.bias[i]);
    // ---- root inputs
    for (int i = tid; i < T * P.obs_feat; i += SM_THREADS) {
        const int gl = i / P.obs_feat, k = i - gl * P.obs_feat;
        const int ggl = tile0 + gl;
        act[P.x_rep + k * T + gl] = ggl < P.G ? P.obs[(size_t)ggl * P.obs_feat + k] : 0.0f;
    }
    if (tree_thread && a == 0) {
        uint32_t m = 0;
        if (active)
            for (int b = 0; b < A; ++b) if (P.legal[(size_t)gg * A + b]) m |= 1u << b;
        sg_legal[g] = m;
        sg_root_tp[g] = active ? P.to_play[gg] : 1;
        sg_rootN[g] = 0; sg_rootW[g] = 0.0f;
        sg_mmin[g] = INFINITY; sg_mmax[g] = -INFINITY;          // MinMaxStats(Inf, -Inf), SelfPlay.jl:251
        sg_leaf_e[g] = 0; sg_leaf_a[g] = 0; sg_vtp[g] = 1; sg_depth[g] = 0;
    }
    __syncthreads();

    // ---- representation (SelfPlay.jl:234): its own schedule, weights loaded once
    {
        float wr[SM_MAX_ROOT][SM_SLOTS][16];
        sm_load<SM_MAX_ROOT>(P.n_root, P.w_root, wr);
        sm_run<T, SM_MAX_ROOT>(P.n_root, wr, rec_root, act, part);
    }
    for (int i = tid; i < T * H; i += SM_THREADS) {     // h -> hidden slot 0 and the prediction input
        const int gl = i / H, k = i - gl * H;
        const float h = act[P.h_out + k * T + gl];
        hid[(size_t)gl * NN * H + k] = h;
        act[P.x_pred + k * T + gl] = h;
    }
    // prediction ‖ dynamics weights: resident for the whole search
    float wr[SM_MAX_SIM][SM_SLOTS][16];
    sm_load<SM_MAX_SIM>(P.n_sim, P.w_sim, wr);
    __syncthreads();
    // prediction(h) for the root (:239); the dynamics half runs on zeros, unused
    sm_run<T, SM_MAX_SIM>(P.n_sim, wr, rec_sim, act, part);

    const uint32_t legal = tree_thread ? sg_legal[g] : 0u;
    if (tree_thread) {   // expand_node!(root, legal, to_play, 0, policy, h) (:245)
        const float prior = double_softmax_prior(a < A ? act[P.p_out + a * T + g] : 0.0f, a, A, legal,
                                                 sg_stage + 16 * g);
        if (active) {
            init_edges(tree, 0, a, A, prior);
            if (a == 0) { tree.nr[0] = 0.0f; tree.ntp[0] = (int8_t)sg_root_tp[g]; }
        }
    }
    __syncthreads();
    if (P.exploration && active && a == 0)                   // add_exploration_noise! (:102-109)
        sm_root_noise(tree.p, legal, A, P.seed, gid, P.rng_step, P.dirichlet_alpha, P.exploration_eps);
    __syncthreads();
    SM_STAMP(0);

    for (int s = 0; s < S; ++s) {
        // ---- select (:256-268)
        if (active) {
            const SelectOut so = select_path(tree, path, sg_rootN[g], sg_root_tp[g], legal, sg_mmin[g], sg_mmax[g],
                                             a, lane, A, P.players, P.discount, P.pbc_tab, P.sqrt_tab, P.seed,
                                             gid, P.rng_step, s);
            if (a == 0) { sg_leaf_e[g] = so.leaf_e; sg_leaf_a[g] = so.leaf_a; sg_vtp[g] = so.vtp; sg_depth[g] = so.depth; }
        }
        __syncthreads();
        SM_STAMP(1);
        // ---- gather: parent h -> prediction input; h *= 2 in place (Q1) -> dynamics input
        for (int i = tid; i < T * H; i += SM_THREADS) {
            const int gl = i / H, k = i - gl * H;
            if (tile0 + gl >= P.G) continue;                  // inactive game of a partial tile
            float* hp = hid + ((size_t)gl * NN + sg_leaf_e[gl]) * H + k;
            const float hv = *hp;
            const float h2 = hv * 2.0f;
            *hp = h2;
            act[P.x_pred + k * T + gl] = hv;
            act[P.x_dyn + k * T + gl] = h2;
        }
        for (int i = tid; i < T * P.plane; i += SM_THREADS) {
            const int gl = i / P.plane, k = i - gl * P.plane;
            if (tile0 + gl >= P.G) continue;
            act[P.x_dyn + (H + k) * T + gl] = P.aval_tab[sg_leaf_a[gl]];
        }
        __syncthreads();
        SM_STAMP(2);
        // ---- prediction(parent.h) ‖ dynamics(2h ⊕ a/|A|)
        sm_run<T, SM_MAX_SIM>(P.n_sim, wr, rec_sim, act, part);
        SM_STAMP(3);
        // ---- expand slot s+1 (:280) + store h'
        const int e_new = s + 1;
        if (tree_thread) {
            const float prior = double_softmax_prior(a < A ? act[P.p_out + a * T + g] : 0.0f, a, A, legal,
                                                     sg_stage + 16 * g);
            if (active) init_edges(tree, e_new, a, A, prior);
        }
        for (int i = tid; i < T * H; i += SM_THREADS) {
            const int gl = i / H, k = i - gl * H;
            hid[((size_t)gl * NN + e_new) * H + k] = act[P.h_out + k * T + gl];
        }
        SM_STAMP(4);
        // ---- backpropagate! (:190-217)
        if (active) {
            const int tl = sg_vtp[g];
            const int depth = sg_depth[g];
            if (a == 0) {
                const int li = sg_leaf_e[g] * A + sg_leaf_a[g];
                tree.nc[li] = (tree.nc[li] & 0xffffu) | ((uint32_t)(e_new + 1) << 16);
                tree.nr[e_new] = mz_post_act(P.r_act, act[P.r_out + g]);
                tree.ntp[e_new] = (int8_t)tl;
                path[2 * depth + 1] = e_new;
            }
            __builtin_amdgcn_wave_barrier();
            int rN = sg_rootN[g];
            float rW = sg_rootW[g], mmin = sg_mmin[g], mmax = sg_mmax[g];
            backup_path(tree, path, depth, mz_post_act(P.v_act, act[P.v_out + g]), tl, A, P.players, P.discount,
                        rN, rW, sg_root_tp[g], mmin, mmax, a);
            if (a == 0) { sg_rootN[g] = rN; sg_rootW[g] = rW; sg_mmin[g] = mmin; sg_mmax[g] = mmax; }
        }
        __syncthreads();
        SM_STAMP(5);
    }

    // ---- store_search_stats! (:115-122) + select_action (:293-306)
    if (active) {
        const bool lg = a < A && ((legal >> a) & 1u);
        const int Nc = lg ? (int)(tree.nc[a] & 0xffffu) : 0;
        const int sum = g16_isum(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        int cnt[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) cnt[b] = __shfl(Nc, b, 16);
        if (a == 0) {
            const int rN = sg_rootN[g];
            P.root_value[gg] = rN == 0 ? 0.0f : sg_rootW[g] / (float)rN;
            const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
            P.action_out[gg] = sm_select_action(cnt, legal, A, P.temperature, r) + 1;
        }
        if (P.dump_tree) {
            TreeView dst = sm_tree_at(P.tree + (size_t)gg * P.tree_game_bytes, E, NN);
            dump_tree(tree, dst, E, NN, a);
        }
    }
#ifdef MZ_STAMPS
    SM_STAMP(6);
    if (threadIdx.x == 0 && P.stamps)
        for (int i = 0; i < 8; ++i) P.stamps[blockIdx.x * 8 + i] = st_acc[i];
#endif
}

extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small1(SmallParams P) { small_body<1>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small2(SmallParams P) { small_body<2>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small4(SmallParams P) { small_body<4>(P); }
