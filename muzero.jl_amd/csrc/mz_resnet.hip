// mz_resnet.hip — the ResNet networks (row a14; Learning.jl:148-255, the
// intended architecture of SURVEY §2.1 Q12) on f32 MFMA, one tile of NG games
// per 256-thread workgroup, activations resident in LDS across all layers.
//
// A layer is a generalised Dense (mz_resnet_params.h).  Each wave takes
// 16x16 output tiles (16 rows of W x 16 columns); a tile's K runs as four
// quarter chains of nq v_mfma_f32_16x16x4_f32 each (k-ordered fmaf chains,
// the canonical order of mz_dot), combined ((p0+p1)+(p2+p3)) + b, then
// BatchNorm in test mode (γ·((t − μ)/√(σ²+ε)) + β with μ = 0, σ² = 1), the
// residual (a block's second conv reads T and overwrites the block input in
// place), and the activation.  Operand maps as mz_mlp_device.h: lane l holds
// A[l&15][l>>4] (pre-packed fragments, one coalesced load per MFMA) and
// B[l>>4][l&15].
#include "mz_mlp_device.h"
#include "mz_resnet_params.h"

__device__ __forceinline__ float rn_act(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

// B(k, n) of one layer for this lane
struct RnCol {
    int n;        // column
    bool ok;      // n < ncols
    int p, g, w, h;
};

__device__ __forceinline__ float rn_b(const RLayer& L, const RnCol& c, int k, int ncols, int NG, int Wb, int P,
                                      const float* lds) {
    if (!c.ok || k >= L.K) return 0.0f;
    if (L.kk == 1) return lds[L.in_off + k * ncols + c.n];
    const int t = reinterpret_cast<const int*>(lds)[L.ktab + k];      // (ch << 8) | (dx+8) << 4 | (dy+8)
    const int ch = t >> 8, dx = ((t >> 4) & 15) - 8, dy = (t & 15) - 8;
    const int sx = c.w + dx, sy = c.h + dy;
    if (sx < 0 || sx >= Wb || sy < 0 || sy >= P / Wb) return 0.0f;
    return lds[L.in_off + ch * ncols + (sx + Wb * sy) * NG + c.g];
}

__device__ void rn_layer(const RLayer& L, const float* __restrict__ Wimg, const float* __restrict__ flat,
                         float* lds, int NG, int Wb, int P, float bn_s) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
    const int ncols = L.spatial ? P * NG : NG;
    const int n_nb = (ncols + 15) >> 4;
    const int NQ = L.nq;
    for (int t = wave; t < L.n_ob * n_nb; t += nwaves) {
        const int ob = t / n_nb, nb = t - ob * n_nb;
        RnCol c;
        c.n = nb * 16 + (lane & 15);
        c.ok = c.n < ncols;
        c.p = c.n / NG; c.g = c.n - c.p * NG;
        c.w = c.p % Wb; c.h = c.p / Wb;
        const float* wb = Wimg + L.w_img + (size_t)ob * (4 * NQ * 64) + lane;
        mz_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
        const int kl = lane >> 4;
        for (int j = 0; j < NQ; ++j) {
            const int k0 = (0 * NQ + j) * 4 + kl, k1 = (1 * NQ + j) * 4 + kl;
            const int k2 = (2 * NQ + j) * 4 + kl, k3 = (3 * NQ + j) * 4 + kl;
            const float b0 = rn_b(L, c, k0, ncols, NG, Wb, P, lds), b1 = rn_b(L, c, k1, ncols, NG, Wb, P, lds);
            const float b2 = rn_b(L, c, k2, ncols, NG, Wb, P, lds), b3 = rn_b(L, c, k3, ncols, NG, Wb, P, lds);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(0 * NQ + j) * 64], b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(1 * NQ + j) * 64], b1, acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(2 * NQ + j) * 64], b2, acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[(3 * NQ + j) * 64], b3, acc3, 0, 0, 0);
        }
        if (!c.ok) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = ob * 16 + kl * 4 + r;
            if (o >= L.cout) continue;
            float d = (acc0[r] + acc1[r]) + (acc2[r] + acc3[r]);
            d = d + flat[L.boff + o];
            if (L.bn) d = flat[L.bnoff + L.cout + o] * ((d - 0.0f) / bn_s) + flat[L.bnoff + o];
            if (L.res_add) d = d + lds[L.res_off + o * ncols + c.n];
            lds[L.out_off + o * ncols + c.n] = rn_act(L.act, d);
        }
    }
}

// the k tables of the layers with a kernel > 1x1 (filled once per launch)
__device__ void rn_fill_ktabs(const RPlan& R, float* lds) {
    for (int i = 0; i < R.n; ++i) {
        const RLayer& L = R.L[i];
        if (L.kk == 1) continue;
        int* tab = reinterpret_cast<int*>(lds) + L.ktab;
        for (int k = threadIdx.x; k < L.K; k += blockDim.x) {
            const int ch = k / L.kk, r = k - ch * L.kk, j = r / L.kw, ii = r - j * L.kw;
            const int dx = (L.kw - 1 - ii) - L.pw, dy = (L.kh - 1 - j) - L.ph;
            tab[k] = (ch << 8) | ((dx + 8) << 4) | (dy + 8);
        }
    }
}

__device__ void rn_run(const RPlan& R, const float* Wimg, const float* flat, float* lds, int NG, int Wb, int P,
                       float bn_s) {
    for (int i = 0; i < R.n; ++i) {
        rn_layer(R.L[i], Wimg, flat, lds, NG, Wb, P, bn_s);
        __syncthreads();
    }
}

// Batched forward of one net (mz_net_forward): x (in_feat, n) -> out0, out1.
extern "C" __global__ __launch_bounds__(256) void mz_rnet_forward_kernel(RNetParams Q) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& R = *Q.plan;
    const int NG = Q.ng, t0 = blockIdx.x * NG;
    rn_fill_ktabs(R, lds);
    for (int i = threadIdx.x; i < R.in_feat * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        lds[R.in_off + i] = t0 + g < Q.n_items ? Q.x[(size_t)(t0 + g) * R.in_feat + f] : 0.0f;
    }
    __syncthreads();
    rn_run(R, Q.Wimg, Q.flat, lds, NG, Q.W, Q.P, Q.bn_s);
    for (int i = threadIdx.x; i < R.out0_n * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        if (t0 + g < Q.n_items) Q.out0[(size_t)(t0 + g) * R.out0_n + f] = lds[R.out0_off + i];
    }
    if (R.out1_n && Q.out1) {
        const int g = threadIdx.x;
        if (g < NG && t0 + g < Q.n_items) {
            float* o = Q.out1 + (size_t)(t0 + g) * R.out1_n;
            const float* x = lds + R.out1_off + g;
            if (Q.softmax1) {                       // NNlib softmax (Learning.jl:225): max, exp, ascending sum
                float m = x[0];
                for (int k = 1; k < R.out1_n; ++k) m = m > x[k * NG] ? m : x[k * NG];
                float s = 0.0f;
                for (int k = 0; k < R.out1_n; ++k) s = s + det_expf(x[k * NG] - m);
                for (int k = 0; k < R.out1_n; ++k) o[k] = det_expf(x[k * NG] - m) / s;
            } else {
                for (int k = 0; k < R.out1_n; ++k) o[k] = x[k * NG];
            }
        }
    }
}

// ================================================================= search
#include "mz_tree_device.h"

__device__ __forceinline__ TreeView rs_tree(const RSearchParams& P, int gg) {
    const int E = (P.S + 1) * P.A, NN = P.S + 1;
    return tree_view(P.tree + (size_t)gg * P.tree_game_bytes, E, NN);
}

// Root (SelfPlay.jl:230-251): representation + prediction of NG games per
// tile, h0 -> hidden slot 0, root expansion with the double softmax (Q3),
// exploration noise, per-game state.
extern "C" __global__ __launch_bounds__(256) void mz_rsearch_root(RSearchParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = P.plans[MZ_NET_REPR];
    const RPlan& Rp = P.plans[MZ_NET_PRED];
    const int NG = P.ng, t0 = blockIdx.x * NG, H = P.H, A = P.A;
    const int nplan = Rr.lds_floats > Rp.lds_floats ? Rr.lds_floats : Rp.lds_floats;
    float* stg = lds + nplan;                       // [16][16] softmax / noise staging
    float* noise = stg + 256;                       // [16][16]
    rn_fill_ktabs(Rr, lds);
    for (int i = threadIdx.x; i < Rr.in_feat * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        lds[Rr.in_off + i] = t0 + g < P.G ? P.obs[(size_t)(t0 + g) * P.obs_feat + f] : 0.0f;
    }
    __syncthreads();
    rn_run(Rr, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s);                    // :234
    for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        if (t0 + g < P.G) P.hid[(size_t)(t0 + g) * (P.S + 1) * H + f] = lds[Rr.out0_off + i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {                  // prediction input = h0
        const int f = i / NG, g = i - f * NG;
        lds[Rp.in_off + i] = t0 + g < P.G ? P.hid[(size_t)(t0 + g) * (P.S + 1) * H + f] : 0.0f;
    }
    __syncthreads();
    rn_run(Rp, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s);                    // :239
    const int gl = threadIdx.x >> 4, a = threadIdx.x & 15, gg = t0 + gl;
    const bool active = gl < NG && gg < P.G;
    if (active) {
        uint32_t legal = 0;
        for (int b = 0; b < A; ++b) if (P.legal[(size_t)gg * A + b]) legal |= 1u << b;
        const uint32_t gid = P.game_offset + (uint32_t)gg;
        TreeView tree = rs_tree(P, gg);
        const float prior = double_softmax_prior(a < A ? lds[Rp.out1_off + a * NG + gl] : 0.0f, a, A, legal,
                                                 stg + 16 * gl);
        init_edges(tree, 0, a, A, prior);                                       // :245
        if (P.exploration) {                                                    // :247-249
            const float nz = root_noise_lane(legal, a, A, P.seed, gid, P.rng_step, P.dirichlet_alpha,
                                             noise + 16 * gl);
            if (a < A && ((legal >> a) & 1u))
                tree.p(a) = tree.p(a) * (1.0f - P.exploration_eps) + nz * P.exploration_eps;
        }
        if (a == 0) {
            int* st = P.gst + (size_t)gg * RG_INTS;
            tree.nr[0] = 0.0f; tree.ntp[0] = (int8_t)P.to_play[gg];
            st[RG_LEGAL] = (int)legal; st[RG_ROOT_TP] = P.to_play[gg];
            st[RG_ROOTN] = 0; st[RG_ROOTW] = __float_as_int(0.0f);
            st[RG_MMIN] = __float_as_int(INFINITY); st[RG_MMAX] = __float_as_int(-INFINITY);   // :251
            st[RG_LEAF_E] = 0; st[RG_LEAF_A] = 0; st[RG_VTP] = 1; st[RG_DEPTH] = 0;
        }
    }
}

// Tree step s: expand + backup of simulation s-1 (s > 0), then select +
// gather for simulation s (s < S), or the search statistics and the action
// (s == S).  16 lanes per game, 16 games per workgroup.
extern "C" __global__ __launch_bounds__(256) void mz_rsearch_tree(RSearchParams P) {
    __shared__ float stg[256];
    const int gl = threadIdx.x >> 4, a = threadIdx.x & 15, lane = threadIdx.x & 63;
    const int gg = blockIdx.x * 16 + gl;
    if (gg >= P.G) return;                          // whole 16-lane groups leave together
    const int A = P.A, H = P.H, S = P.S, PS = 2 * (S + 2);
    int* st = P.gst + (size_t)gg * RG_INTS;
    int* path = P.path + (size_t)gg * PS;
    TreeView tree = rs_tree(P, gg);
    const uint32_t legal = (uint32_t)st[RG_LEGAL];
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    if (P.s > 0) {
        const int e_new = P.s;                      // the node simulation s-1 expanded (:280)
        const float prior = double_softmax_prior(a < A ? P.o_logit[(size_t)gg * A + a] : 0.0f, a, A, legal,
                                                 stg + 16 * gl);
        init_edges(tree, e_new, a, A, prior);
        const int tl = st[RG_VTP], depth = st[RG_DEPTH];
        if (a == 0) {
            const int li = st[RG_LEAF_E] * A + st[RG_LEAF_A];
            tree.nc(li) = (tree.nc(li) & 0xffffu) | ((uint32_t)(e_new + 1) << 16);
            tree.nr[e_new] = P.o_r[gg];
            tree.ntp[e_new] = (int8_t)tl;
            path[2 * depth + 1] = e_new;
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        int rN = st[RG_ROOTN];
        float rW = __int_as_float(st[RG_ROOTW]);
        float mmin = __int_as_float(st[RG_MMIN]), mmax = __int_as_float(st[RG_MMAX]);
        backup_path(tree, path, depth, P.o_v[gg], tl, A, P.players, P.discount, rN, rW, st[RG_ROOT_TP], mmin,
                    mmax, a);                                                   // :281
        __builtin_amdgcn_wave_barrier();
        if (a == 0) {
            st[RG_ROOTN] = rN; st[RG_ROOTW] = __float_as_int(rW);
            st[RG_MMIN] = __float_as_int(mmin); st[RG_MMAX] = __float_as_int(mmax);
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
    if (P.s < S) {
        const SelectOut so = select_path<false>(tree, path, st[RG_ROOTN], st[RG_ROOT_TP], legal,
                                                __int_as_float(st[RG_MMIN]), __int_as_float(st[RG_MMAX]), a, lane,
                                                A, P.players, P.discount, nullptr, P.pbc_tab, P.sqrt_tab, P.seed,
                                                gid, P.rng_step, P.s);                    // :256-268
        if (a == 0) {
            st[RG_LEAF_E] = so.leaf_e; st[RG_LEAF_A] = so.leaf_a; st[RG_VTP] = so.vtp; st[RG_DEPTH] = so.depth;
        }
        // parent h -> prediction input; h *= 2 in place (Q1), read by the dynamics launch
        float* hp = P.hid + ((size_t)gg * (S + 1) + so.leaf_e) * H;
        float* xp = P.x_pred + (size_t)gg * H;
        for (int k = a; k < H; k += 16) {
            const float hv = hp[k];
            xp[k] = hv;
            hp[k] = hv * 2.0f;
        }
    } else {                                        // store_search_stats! (:115-122) + select_action (:293-306)
        const bool lg = a < A && ((legal >> a) & 1u);
        const int Nc = lg ? (int)(tree.nc(a) & 0xffffu) : 0;
        const int sum = g16_isum(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        int cnt[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) cnt[b] = __shfl(Nc, b, 16);
        if (a == 0) {
            const int rN = st[RG_ROOTN];
            P.root_value[gg] = rN == 0 ? 0.0f : __int_as_float(st[RG_ROOTW]) / (float)rN;
            const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
            P.action_out[gg] = select_action_dev(cnt, legal, A, P.temperature, r) + 1;
        }
    }
}

// Networks of simulation s: blockIdx.y = 0 prediction(parent h), 1 dynamics
// (2h ⊕ a/|A|, Q1) writing h' into hidden slot s+1.
extern "C" __global__ __launch_bounds__(256) void mz_rsearch_nets(RSearchParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int net = blockIdx.y == 0 ? MZ_NET_PRED : MZ_NET_DYN;
    const RPlan& R = P.plans[net];
    const int NG = P.ng, t0 = blockIdx.x * NG, H = P.H, S = P.S;
    rn_fill_ktabs(R, lds);
    for (int i = threadIdx.x; i < R.in_feat * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG, gg = t0 + g;
        float v = 0.0f;
        if (gg < P.G) {
            const int* st = P.gst + (size_t)gg * RG_INTS;
            if (net == MZ_NET_PRED) v = P.x_pred[(size_t)gg * H + f];
            else if (f < H) v = P.hid[((size_t)gg * (S + 1) + st[RG_LEAF_E]) * H + f];
            else v = P.aval_tab[st[RG_LEAF_A]];
        }
        lds[R.in_off + i] = v;
    }
    __syncthreads();
    rn_run(R, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s);
    if (net == MZ_NET_PRED) {
        for (int i = threadIdx.x; i < (1 + P.A) * NG; i += blockDim.x) {
            const int r = i / NG, g = i - r * NG, gg = t0 + g;
            if (gg >= P.G) continue;
            if (r == 0) P.o_v[gg] = lds[R.out0_off + g];
            else P.o_logit[(size_t)gg * P.A + (r - 1)] = lds[R.out1_off + (r - 1) * NG + g];
        }
    } else {
        for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {
            const int f = i / NG, g = i - f * NG, gg = t0 + g;
            if (gg < P.G) P.hid[((size_t)gg * (S + 1) + P.s + 1) * H + f] = lds[R.out0_off + i];
        }
        if (threadIdx.x < NG && t0 + (int)threadIdx.x < P.G) P.o_r[t0 + threadIdx.x] = lds[R.out1_off + threadIdx.x];
    }
}

// ================================================================ learner
// Forward unroll of the learner (Learning.jl:347-370): representation, then
// for i = 1..K prediction(h_{i-1}) -> step i (step 0 is the same prediction of
// h0, written once for both), dynamics(2h ⊕ a_i/|A|) -> h_i, r_i; r_0 = 0.
extern "C" __global__ __launch_bounds__(256) void mz_runroll_kernel(RUnrollParams U) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = U.plans[MZ_NET_REPR];
    const RPlan& Rp = U.plans[MZ_NET_PRED];
    const RPlan& Rd = U.plans[MZ_NET_DYN];
    const int NG = U.ng, t0 = blockIdx.x * NG, H = U.H, A = U.A, K1 = U.K + 1;
    rn_fill_ktabs(Rr, lds);
    for (int i = threadIdx.x; i < Rr.in_feat * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        lds[Rr.in_off + i] = t0 + g < U.B ? U.obs[(size_t)(t0 + g) * U.obs_feat + f] : 0.0f;
    }
    __syncthreads();
    rn_run(Rr, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                     // :347
    for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {
        const int f = i / NG, g = i - f * NG;
        if (t0 + g < U.B) U.hs[(size_t)(t0 + g) * H + f] = lds[Rr.out0_off + i];
    }
    if (threadIdx.x < NG && t0 + (int)threadIdx.x < U.B) U.pr[(size_t)(t0 + threadIdx.x) * K1] = 0.0f;
    const int ns = U.K > 0 ? U.K : 1;              // K = 0: the prediction of h0 alone
    for (int s = 1; s <= ns; ++s) {
        __syncthreads();
        rn_fill_ktabs(Rp, lds);
        for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {
            const int f = i / NG, g = i - f * NG;
            lds[Rp.in_off + i] = t0 + g < U.B ? U.hs[(size_t)(t0 + g) * H + f] : 0.0f;
        }
        __syncthreads();
        rn_run(Rp, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                 // :351 / :356
        for (int i = threadIdx.x; i < (1 + A) * NG; i += blockDim.x) {
            const int r = i / NG, g = i - r * NG, b = t0 + g;
            if (b >= U.B) continue;
            const float v = r == 0 ? lds[Rp.out0_off + g] : lds[Rp.out1_off + (r - 1) * NG + g];
            for (int j = s == 1 ? 0 : s; j <= (s <= U.K ? s : 0); ++j) {
                if (r == 0) U.pv[(size_t)b * K1 + j] = v;
                else U.pp[((size_t)b * K1 + j) * A + (r - 1)] = v;
            }
        }
        if (s > U.K) break;
        __syncthreads();
        rn_fill_ktabs(Rd, lds);
        for (int i = threadIdx.x; i < Rd.in_feat * NG; i += blockDim.x) {     // make_dynamics_input (:293-304)
            const int f = i / NG, g = i - f * NG, b = t0 + g;
            float v = 0.0f;
            if (b < U.B) v = f < H ? U.hs[(size_t)b * H + f] * 2.0f : U.actions[(size_t)b * K1 + (s - 1)] / (float)A;
            lds[Rd.in_off + i] = v;
        }
        __syncthreads();
        rn_run(Rd, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                 // :362
        for (int i = threadIdx.x; i < H * NG; i += blockDim.x) {
            const int f = i / NG, g = i - f * NG;
            if (t0 + g < U.B) U.hs[(size_t)(t0 + g) * H + f] = lds[Rd.out0_off + i];
        }
        if (threadIdx.x < NG && t0 + (int)threadIdx.x < U.B)
            U.pr[(size_t)(t0 + threadIdx.x) * K1 + s] = lds[Rd.out1_off + threadIdx.x];
    }
}
