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
