// mz_search.hip — batched MCTS (run_mcts + select_action + store_search_stats!)
// as ONE persistent kernel launch per move (reference: src/SelfPlay.jl:230-306).
//
// Workgroup = 256 threads = a tile of 16 games.  The kernel runs the root
// inference (representation + prediction, :234,:239), the root expansion and
// Dirichlet noise (:245-249), then loops over the S simulations (:254-283)
// with no grid-wide synchronisation — games are independent:
//
//   select   (:261-268)  thread (g, a) = (tid>>4, tid&15): 16 lanes per game,
//                        one child slot per lane; pUCT in f64 (Q5), argmax and
//                        tie count by 16-lane shuffles/ballot, Philox tie-break;
//   gather   (:271-273)  parent hidden state h -> prediction input; h *= 2 in
//                        place in HBM (Q1) -> dynamics input with the a/|A| plane;
//   nets     (:271,:275) prediction ‖ dynamics as one 8-stage MFMA plan;
//   expand   (:280)      double softmax (Q3) over the root's legal set (Q4);
//   backup   (:281)      Q7 along the recorded path, per-game min-max stats.
//
// Tree storage is structure-of-arrays in HBM: edges [G][S+1][A] (N, W, P, R,
// child slot), node to_play [G][S+1], hidden [G][S+1][H].  Expanded-node slot
// e = 0 is the root, e = s+1 the node expanded by simulation s.
#include "mz_mlp_device.h"

__device__ __forceinline__ float g16_max(float v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {
        float t = __shfl_xor(v, o, 16);
        v = v > t ? v : t;
    }
    return v;
}

__device__ __forceinline__ int g16_isum(int v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}

// sequential (ascending) f32 sum of lanes 0..n-1 of the 16-lane group; every
// lane returns the same value (the oracle's `s = s + y[i]` loop order).
__device__ __forceinline__ float g16_seqsum(float v, int n) {
    float s = 0.0f;
    for (int b = 0; b < n; ++b) s = s + __shfl(v, b, 16);
    return s;
}

__device__ __forceinline__ int nth_set_bit(uint32_t m, int k) {
    for (int i = 0; i < k; ++i) m &= m - 1;
    return __builtin_ctz(m);
}

// expand_node! (SelfPlay.jl:88-96) for the 16-lane group of game g: the
// policy head's softmax over all A logits (Learning.jl:114) and then the
// softmax over the legal entries (:89, Q3).  Returns this lane's prior.
__device__ __forceinline__ float double_softmax_prior(const float* act, int p_out, int g, int a, int A,
                                                      uint32_t legal) {
    const bool in = a < A;
    const float logit = in ? act[p_out + a * 16 + g] : -INFINITY;
    const float m = g16_max(logit);
    const float ex = in ? det_expf(logit - m) : 0.0f;
    const float s = g16_seqsum(ex, A);
    const float prob = in ? ex / s : 0.0f;
    const bool lg = in && ((legal >> a) & 1u);
    const float m2 = g16_max(lg ? prob : -INFINITY);
    const float e2 = lg ? det_expf(prob - m2) : 0.0f;
    const float s2 = g16_seqsum(e2, A);     // illegal lanes add +0: same as the legal-only sum
    return lg ? e2 / s2 : 0.0f;
}

// select_action (SelfPlay.jl:293-306): same rule as the oracle.
__device__ int select_action_dev(const int* cnt, uint32_t legal, int A, float temperature, uint32_t r) {
    int acts[16], c[16], n = 0;
    for (int a = 0; a < A; ++a) if ((legal >> a) & 1u) { acts[n] = a; c[n] = cnt[a]; ++n; }
    if (temperature == 0.0f) {
        int best = 0;
        for (int i = 1; i < n; ++i) if (c[i] > c[best]) best = i;
        return acts[best];
    }
    if (isinf(temperature)) return acts[mz_rng_below(r, (uint32_t)n)];
    if (temperature == 1.0f) {
        uint32_t tot = 0;
        for (int i = 0; i < n; ++i) tot += (uint32_t)c[i];
        if (tot == 0) return acts[mz_rng_below(r, (uint32_t)n)];
        uint32_t t = mz_rng_below(r, tot), cum = 0;
        for (int i = 0; i < n; ++i) { cum += (uint32_t)c[i]; if (cum > t) return acts[i]; }
        return acts[n - 1];
    }
    float e = 1.0f / temperature;
    float w[16], s = 0.0f;
    for (int i = 0; i < n; ++i) {
        w[i] = c[i] > 0 ? (float)det_exp(det_log((double)c[i]) * (double)e) : 0.0f;
        s = s + w[i];
    }
    float u = (float)(r >> 8) * 5.9604644775390625e-08f * s;
    float cum = 0.0f;
    for (int i = 0; i < n; ++i) { cum = cum + w[i]; if (cum > u) return acts[i]; }
    return acts[n - 1];
}

extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_search_kernel(SearchParams P) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* act = smem;
    int* si = reinterpret_cast<int*>(smem + P.lay.total);
    // per-game scratch (16 entries each)
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
    int* sg_path = si + 160;                 // [16][S+2]: (e << 8) | a

    const int tid = threadIdx.x, lane = tid & 63;
    const int g = tid >> 4, a = tid & 15;
    const int A = P.A, S = P.S, H = P.H;
    const int tile0 = blockIdx.x * MZ_TILE;
    const int gg = tile0 + g;
    const bool active = gg < P.G;
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    const size_t tbase = (size_t)gg * P.tree_stride;          // edges of game gg
    const int PS = S + 2;

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

    // ---- representation (:234) -> h_out, prediction(h) (:239) -> v_out, p_out
    run_plan(P.plan_root, P.Wp, P.Bp, act);

    for (int i = tid; i < MZ_TILE * H; i += blockDim.x) {
        const int gl = i / H, k = i - gl * H;
        const int ggl = tile0 + gl;
        if (ggl < P.G) P.hid[(size_t)ggl * (S + 1) * H + k] = act[P.lay.h_out + k * 16 + gl];
    }
    const uint32_t legal = sg_legal[g];
    const bool lg = a < A && ((legal >> a) & 1u);
    {   // expand_node!(root, legal, to_play, 0, policy, h) (:245)
        const float prior = double_softmax_prior(act, P.lay.p_out, g, a, A, legal);
        if (active && a < A) {
            const size_t idx = tbase + a;
            P.eN[idx] = 0; P.eW[idx] = 0.0f; P.eP[idx] = prior; P.eR[idx] = 0.0f; P.eC[idx] = -1;
        }
        if (active && a == 0) P.ntp[(size_t)gg * (S + 1)] = sg_root_tp[g];
    }
    __syncthreads();
    if (P.exploration && active && a == 0) {                 // add_exploration_noise! (:102-109)
        int n = __builtin_popcount(legal);
        float noise[MZ_MAX_ACTIONS];
        mz_dirichlet(P.seed, gid, P.rng_step, n, P.dirichlet_alpha, noise);
        const float one_m = 1.0f - P.exploration_eps;
        int i = 0;
        for (int b = 0; b < A; ++b) if ((legal >> b) & 1u) {
            const size_t idx = tbase + b;
            P.eP[idx] = P.eP[idx] * one_m + noise[i] * P.exploration_eps;
            ++i;
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- simulations
    for (int s = 0; s < S; ++s) {
        // ---- select (:256-268)
        if (active) {
            int e = 0, Np = sg_rootN[g], depth = 0, vtp = sg_root_tp[g];
            const float mmin = sg_mmin[g], mmax = sg_mmax[g];
            for (;;) {
                const size_t idx = tbase + (size_t)e * A + a;
                int Nc = 0, Cc = -1;
                float u = -INFINITY;
                if (lg) {
                    Nc = P.eN[idx]; Cc = P.eC[idx];
                    const float Wc = P.eW[idx], Pc = P.eP[idx], Rc = P.eR[idx];
                    // ucb_score (:171-184), Q5
                    const double pb_c = P.pbc_tab[Np] * (P.sqrt_tab[Np] / (double)(Nc + 1));
                    const double prior_score = pb_c * (double)Pc;
                    float vs = 0.0f;
                    if (Nc > 0) {
                        const float q = Wc / (float)Nc;
                        const float t = P.players == 1 ? P.discount * q : P.discount * (-q);
                        const float v = Rc + t;
                        vs = mmax > mmin ? (v - mmin) / (mmax - mmin) : v;
                    }
                    u = (float)(prior_score + (double)vs);
                }
                const float m = g16_max(u);
                const uint64_t bal = __ballot(lg && u == m);
                const uint32_t mask = (uint32_t)(bal >> (lane & 48)) & 0xffffu;
                const int nt = __builtin_popcount(mask);
                depth += 1;
                const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_TIE, gid, P.rng_step,
                                              ((uint32_t)s << 12) | (uint32_t)depth);
                const int ach = nth_set_bit(mask, (int)mz_rng_below(r, (uint32_t)nt));
                const int Cch = __shfl(Cc, ach, 16);
                const int Nch = __shfl(Nc, ach, 16);
                if (a == 0) sg_path[g * PS + depth] = (e << 8) | ach;
                vtp = (vtp % P.players) + 1;                        // mod1(vtp+1, |players|)
                if (Cch < 0) {
                    if (a == 0) { sg_leaf_e[g] = e; sg_leaf_a[g] = ach; sg_vtp[g] = vtp; sg_depth[g] = depth; }
                    break;
                }
                e = Cch; Np = Nch;
            }
        }
        __syncthreads();

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

        // ---- prediction(parent.h) ‖ dynamics(2h ⊕ a/|A|)
        run_plan(P.plan_sim, P.Wp, P.Bp, act);

        // ---- expand the leaf as slot s+1 (:280)
        const int e_new = s + 1;
        {
            const float prior = double_softmax_prior(act, P.lay.p_out, g, a, A, legal);
            if (active && a < A) {
                const size_t idx = tbase + (size_t)e_new * A + a;
                P.eN[idx] = 0; P.eW[idx] = 0.0f; P.eP[idx] = prior; P.eR[idx] = 0.0f; P.eC[idx] = -1;
            }
        }
        for (int i = tid; i < MZ_TILE * H; i += blockDim.x) {
            const int gl = i / H, k = i - gl * H;
            const int ggl = tile0 + gl;
            if (ggl < P.G) P.hid[((size_t)ggl * (S + 1) + e_new) * H + k] = act[P.lay.h_out + k * 16 + gl];
        }
        // ---- backpropagate! (:190-217), one lane per game
        if (active && a == 0) {
            const int tl = sg_vtp[g];
            const size_t leaf = tbase + (size_t)sg_leaf_e[g] * A + sg_leaf_a[g];
            P.eC[leaf] = e_new;
            P.eR[leaf] = act[P.lay.r_out + g];
            P.ntp[(size_t)gg * (S + 1) + e_new] = tl;
            float v = act[P.lay.v_out + g];
            float mmin = sg_mmin[g], mmax = sg_mmax[g];
            const float disc = P.discount;
            for (int d = sg_depth[g]; d >= 0; --d) {
                int N; float W, R; int tp; size_t idx = 0;
                if (d > 0) {
                    const int pe = sg_path[g * PS + d];
                    idx = tbase + (size_t)(pe >> 8) * A + (pe & 255);
                    N = P.eN[idx]; W = P.eW[idx]; R = P.eR[idx];
                    tp = P.ntp[(size_t)gg * (S + 1) + P.eC[idx]];
                } else {
                    N = sg_rootN[g]; W = sg_rootW[g]; R = 0.0f; tp = sg_root_tp[g];
                }
                if (P.players == 1) {
                    W = W + v; N += 1;
                    const float upd = R + disc * (W / (float)N);
                    mmin = mmin < upd ? mmin : upd; mmax = mmax > upd ? mmax : upd;
                    v = R + disc * v;
                } else {
                    W = tp == tl ? W + v : W - v;
                    N += 1;
                    const float upd = R + disc * (W / (float)N);
                    mmin = mmin < upd ? mmin : upd; mmax = mmax > upd ? mmax : upd;
                    v = tp == tl ? -R : R + disc * v;
                }
                if (d > 0) { P.eN[idx] = N; P.eW[idx] = W; }
                else { sg_rootN[g] = N; sg_rootW[g] = W; }
            }
            sg_mmin[g] = mmin; sg_mmax[g] = mmax;
        }
        __syncthreads();
    }

    // ---- store_search_stats! (:115-122) + select_action (:293-306)
    if (active) {
        const int Nc = lg ? P.eN[tbase + a] : 0;
        const int sum = g16_isum(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        int cnt[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) cnt[b] = __shfl(Nc, b, 16);
        if (a == 0) {
            const int rN = sg_rootN[g];
            P.root_value[gg] = rN == 0 ? 0.0f : sg_rootW[g] / (float)rN;
            const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
            P.action_out[gg] = select_action_dev(cnt, legal, A, P.temperature, r) + 1;
        }
    }
}
