// mz_downsample.hip — the downsampler of the ResNet representation
// (ResNetHP.downsample, src/Learning.jl:175-187) for BASELINE configs[4]
// (84x84x4 observations): one workgroup per item runs every layer of the
// DsPlan with the activations in LDS; the result (6, 6, 2C) goes to HBM,
// where the representation's tail (mz_rsearch_root / mz_runroll_kernel /
// mz_rnet_forward_kernel) reads it as its input.  The 3x3 convs run one
// thread per output position with compile-time taps (ds_conv3).
//
// Numerics = oracle/mz_oracle.c conv_fwd / pool_fwd bit for bit: each output
// is the canonical dot (four k-quarter fmaf chains of length 4⌈K/16⌉ over
// k = i + kw·j + kw·kh·c, ((p0+p1)+(p2+p3))) + bias, then BatchNorm
// γ·((t - 0)/s) + β, the block input, the activation; MeanPool sums the
// in-board window rows outer / columns inner and multiplies by f32(1/9).
// The work is small (≈ 3.3 M MACs per item, once per move) next to the
// S simulations of the search; what bounds it is the latency of one item's
// 20 dependent layers.  The 8-channel convs run as f32 MFMA implicit GEMMs
// (ds_conv_mfma, since round 5); the 4-channel convs stay on the VALU
// (ds_conv3: 16x16 MFMA tiles would be ¾ padding), each position's taps
// loaded once, in one batch, and reused for every output channel.
#include <hip/hip_runtime.h>
#include "mz_internal.h"
#include "mz_resnet_params.h"

__device__ __forceinline__ float ds_act(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

// One 3x3 conv (Flux cross-correlation with the kernel flipped, pad 1, stride
// S) of the downsampler, CIN -> COUT channels, every tap index compile-time.
// One thread per output position: its K = 9·CIN taps are loaded once (all
// issued before any fma), then all COUT outputs of the position are formed
// from them, each as the canonical four k-quarter fmaf chains (kq = 4⌈K/16⌉,
// k = i + 3j + 9c) — the oracle's conv_fwd order, bit for bit.  The weights
// and biases are wave-uniform: scalar loads, SGPR operands of the fmas.
typedef __attribute__((address_space(3))) float* ds_lptr;          // LDS view
typedef float ds_f32x4 __attribute__((ext_vector_type(4)));

// One 3x3 conv (Flux cross-correlation with the kernel flipped, pad 1, stride
// S), CIN -> COUT <= 16 channels, LDS to LDS, as an implicit GEMM on f32 MFMA
// 16x16x4: A = W (rows = output channels, zero beyond COUT), B = the taps of 16
// output positions, K = 9·CIN in the canonical four k-quarters of kq =
// 4⌈K/16⌉ (k = i + 3j + 9c), each quarter one accumulator chain of kq/4 MFMAs
// — a k-ordered fmaf chain from +0, bit for bit the oracle's conv_fwd dot
// (mz_mlp_device.h; the steps past K add +0 products to a sum that is never
// -0).  Then ((p0 + p1) + (p2 + p3)) + b, BatchNorm, the residual, relu.
// Operands: lane l holds A[co = l & 15][k = 4s + (l >> 4)] (its weights of the
// layer, read once from the packed parameters in LDS) and B[k][position
// l & 15] (one LDS read per step, a clamped index, zero outside the board);
// D: lane l holds channels 4(l >> 4) + r of position l & 15.  A wave takes
// 16-position tiles in turn.
template <int CIN, int COUT, int S>
__device__ __forceinline__ void ds_conv_mfma(const DsLayer& L, ds_lptr in, ds_lptr out, ds_lptr res, ds_lptr pw,
                                             float bn_s) {
    constexpr int K = 9 * CIN, NQ = (K + 15) / 16, KQ = 4 * NQ, NS = 4 * NQ;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int g = lane >> 4, col = lane & 15;
    const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Po = Wo * L.Ho, Pi = Wi * Hi;
    const bool bn = L.bn != 0, relu = L.act == MZ_ACT_RELU, has_res = L.res_add != 0;
    float wr[NS];
    int toff[NS], tdx[NS], tdy[NS];                     // per step: tap offset, dx, dy (k >= K: dx = 4096, off-board)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int q = s / NQ, j = s - q * NQ, k = q * KQ + 4 * j + g;
        const bool kin = k < K;
        const int c = k / 9, jj = (k / 3) % 3, ii = k % 3, dx = 1 - ii, dy = 1 - jj;
        wr[s] = kin && col < COUT ? pw[K * col + k] : 0.0f;
        toff[s] = c * Pi + dy * Wi + dx;
        tdx[s] = kin ? dx : 4096;
        tdy[s] = dy;
    }
    float bias[4], gam[4], bet[4];                      // channels 4g + r of this lane's outputs
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int co = 4 * g + r, cc = co < COUT ? co : 0;
        bias[r] = pw[K * COUT + cc];
        gam[r] = bn ? pw[K * COUT + 2 * COUT + cc] : 1.0f;
        bet[r] = bn ? pw[K * COUT + COUT + cc] : 0.0f;
    }
    const int ntile = (Po + 15) >> 4;
    for (int tile = wave; tile < ntile; tile += nw) {
        const int p = tile * 16 + col;
        const bool pin = p < Po;
        const int pp = pin ? p : 0, oh = pp / Wo, ow = pp - oh * Wo;
        const int sx0 = S * ow, sy0 = S * oh, base = sy0 * Wi + sx0;
        float x[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {                  // every tap load first; branch-free (bitwise tests, a
            const int sx = sx0 + tdx[s], sy = sy0 + tdy[s];   // clamped index, a select): no per-tap control flow
            const bool ok = pin & ((unsigned)sx < (unsigned)Wi) & ((unsigned)sy < (unsigned)Hi);
            const float v = in[ok ? base + toff[s] : 0];
            x[s] = ok ? v : 0.0f;
        }
        ds_f32x4 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = ds_f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int j = 0; j < NQ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int s = q * NQ + j;
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s], x[s], acc[q], 0, 0, 0);
            }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = 4 * g + r;
            if (co < COUT && pin) {
                float t = ((acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r])) + bias[r];
                if (bn) t = gam[r] * ((t - 0.0f) / bn_s) + bet[r];
                const int o = co * Po + p;
                if (has_res) t = t + res[o];
                out[o] = relu ? mz_relu(t) : t;
            }
        }
    }
}

// The same conv on the VALU, one thread per output position: its K taps loaded
// once (branch-free), then all COUT outputs from them as the canonical four
// k-quarter fmaf chains; the weights are wave-uniform LDS reads (broadcasts).
// For the 4-channel layers, whose MFMA tiles would be 3/4 padding rows.
template <int CIN, int COUT, int S>
__device__ __forceinline__ void ds_conv_valu(const DsLayer& L, ds_lptr in, ds_lptr out, ds_lptr res, ds_lptr pw,
                                             float bn_s) {
    constexpr int K = 9 * CIN, KQ = 4 * ((K + 15) / 16);
    const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Po = Wo * L.Ho, Pi = Wi * Hi;
    const bool bn = L.bn != 0, relu = L.act == MZ_ACT_RELU, has_res = L.res_add != 0;
    // two positions per pass (p, p + blockDim): each weight read (an LDS
    // broadcast) feeds both positions' chains, and one position's taps load
    // under the other's fmas (a position past the layer computes on zeros,
    // stores nothing)
    const int nt = blockDim.x, pe = Po;
    for (int pa = (int)threadIdx.x; pa < pe; pa += 2 * nt) {
        asm volatile("" ::: "memory");                  // the weights re-read per pass, not K·COUT live values
        int pp[2];
        bool pin[2];
        float x[2][K];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            pp[h] = pa + h * nt;
            pin[h] = pp[h] < pe;
            const int pc = pin[h] ? pp[h] : pa, oh = pc / Wo, ow = pc - oh * Wo;
            bool okx[3], oky[3];
#pragma unroll
            for (int t = 0; t < 3; ++t) {               // tap i (j): dx (dy) = 1 - i (1 - j)
                okx[t] = pin[h] & ((unsigned)(S * ow + 1 - t) < (unsigned)Wi);
                oky[t] = (unsigned)(S * oh + 1 - t) < (unsigned)Hi;
            }
            const int base = (S * oh) * Wi + S * ow;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = k % 3, j = (k / 3) % 3, c = k / 9;
                const bool ok = okx[i] & oky[j];
                const float v = in[ok ? base + c * Pi + (1 - j) * Wi + (1 - i) : 0];
                x[h][k] = ok ? v : 0.0f;
            }
        }
#pragma unroll
        for (int co = 0; co < COUT; ++co) {
            float part[2][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
                for (int k = q * KQ; k < (q + 1) * KQ && k < K; ++k) {
                    const float wk = pw[K * co + k];
                    a0 = __builtin_fmaf(wk, x[0][k], a0);
                    a1 = __builtin_fmaf(wk, x[1][k], a1);
                }
                part[0][q] = a0; part[1][q] = a1;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!pin[h]) continue;
                float t = ((part[h][0] + part[h][1]) + (part[h][2] + part[h][3])) + pw[K * COUT + co];
                if (bn) t = pw[K * COUT + 2 * COUT + co] * ((t - 0.0f) / bn_s) + pw[K * COUT + COUT + co];
                const int o = co * Po + pp[h];
                if (has_res) t = t + res[o];
                out[o] = relu ? mz_relu(t) : t;
            }
        }
    }
}

// The generic layer (any kernel size / channel count): one thread per output,
// the taps through the LDS offset tables kt / kd, the same canonical order
__device__ __forceinline__ void ds_conv_generic(const DsLayer& L, const float* in, float* out, const float* res,
                                                const float* flat, float bn_s, float* yg, float* wl, int* kt,
                                                int* kd) {
    const int tid = threadIdx.x, Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Ho = L.Ho, Pi = Wi * Hi, Po = Wo * Ho;
    const int K = L.kw * L.kh * L.cin;
    for (int i = tid; i < K * L.cout; i += blockDim.x) wl[i] = flat[L.woff + i];
    for (int k = tid; k < K; k += blockDim.x) {
        const int i = k % L.kw, j = (k / L.kw) % L.kh, c = k / (L.kw * L.kh);
        const int dx = (L.kw - 1 - i) - L.pw, dy = (L.kh - 1 - j) - L.ph;   // Flux: kernel flipped
        kt[k] = c * Pi + dy * Wi + dx;
        kd[k] = (dx + 8) | ((dy + 8) << 4);
    }
    __syncthreads();
    const int kq = 4 * ((K + 15) / 16);
    for (int o = tid; o < L.cout * Po; o += blockDim.x) {
        const int co = o / Po, p = o - co * Po;
        const int oh = p / Wo, ow = p - oh * Wo;
        const int sx0 = L.stride * ow, sy0 = L.stride * oh, base = sx0 + Wi * sy0;
        const float* w = wl + K * co;
        float part[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float acc = 0.0f;
            const int k1 = (q + 1) * kq < K ? (q + 1) * kq : K;
            for (int k = q * kq; k < k1; ++k) {
                const int d = kd[k];
                const int sx = sx0 + (d & 15) - 8, sy = sy0 + (d >> 4) - 8;
                const bool inb = sx >= 0 && sx < Wi && sy >= 0 && sy < Hi;
                const float xv = inb ? in[base + kt[k]] : 0.0f;
                acc = __builtin_fmaf(w[k], xv, acc);
            }
            part[q] = acc;
        }
        float t = ((part[0] + part[1]) + (part[2] + part[3])) + flat[L.boff + co];
        if (L.bn) t = flat[L.bnoff + L.cout + co] * ((t - 0.0f) / bn_s) + flat[L.bnoff + co];
        if (res) t = t + res[o];
        t = ds_act(L.act, t);
        if (out) out[o] = t;
        else yg[o] = t;
    }
}

// MeanPool (no flip), padding counted: the window rows outer / columns inner,
// times f32(1/9); LDS input, output to LDS or (the last layer) to HBM
__device__ __forceinline__ void ds_pool(const DsLayer& L, ds_lptr in, ds_lptr out, float* yg) {
    const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Po = Wo * L.Ho, Pi = Wi * Hi;
    const float inv = 1.0f / (float)(L.kw * L.kh);
    const bool lds_out = L.out_buf >= 0;
    for (int o = threadIdx.x; o < L.cout * Po; o += blockDim.x) {
        const int c = o / Po, p = o - c * Po;
        const int oh = p / Wo, ow = p - oh * Wo;
        float m = 0.0f;
        for (int j = 0; j < L.kh; ++j)
            for (int i = 0; i < L.kw; ++i) {
                const int sx = L.stride * ow + i - L.pw, sy = L.stride * oh + j - L.ph;
                const bool ok = ((unsigned)sx < (unsigned)Wi) & ((unsigned)sy < (unsigned)Hi);
                const float v = in[ok ? sx + Wi * sy + Pi * c : 0];
                if (ok) m = m + v;                          // (only in-board terms: the oracle's sum)
            }
        const float t = inv * m;
        if (lds_out) out[o] = t;
        else yg[o] = t;
    }
}

#ifdef __HIP_DEVICE_COMPILE__
typedef const __attribute__((address_space(4))) DsPlan* ds_plan_cptr;   // the plan by scalar loads
#else
typedef const DsPlan* ds_plan_cptr;                                      // (the kernel's host pass)
#endif

extern "C" __global__ __launch_bounds__(DS_THREADS) void mz_downsample_kernel(DsParams Q) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // the plan is read-only for the whole launch: through the constant address
    // space its fields are scalar loads (as a generic pointer that a store could
    // alias, each layer re-read it with vector loads and a full wait)
    const ds_plan_cptr Dp = (ds_plan_cptr)Q.plan;
    const auto& D = *Dp;
    const int item = blockIdx.x, tid = threadIdx.x;
    const int nl = D.n, bf = D.buf_floats, stage = D.stage_in, lf = D.lds_floats, pn_max = D.pn_max;
    float* buf[2] = {lds, lds + bf};
    float* pwl = lds + lf;                                   // [pn_max] layer 0's packed parameters
    float* wl = pwl + pn_max;                                // [cout][K] weights of the current conv (generic)
    int* kt = reinterpret_cast<int*>(wl + D.w_floats);       // [K]: c·Pi + dy·Wi + dx
    int* kd = kt + 256;                                      // [K]: (dx + 8) | (dy + 8) << 4
    float* pall = lds + 2 * bf;                              // after layer 0: every conv's parameters
    const float* xg = Q.x + (size_t)item * D.in_feat;
    float* yg = Q.y + (size_t)item * D.out_feat;
    const int w0 = D.L[0].woff;
    const float* flat = Q.per_step > 0 ? Q.flat + (size_t)(item / Q.per_step) * Q.flat_stride : Q.flat;
    // (LDS pointers as address-space-3 values: offset 0, buffer 0, is that
    // space's null, so nothing below tests them for null)
    const ds_lptr lb0 = (ds_lptr)buf[0], lb1 = (ds_lptr)buf[1];
#ifdef MZ_STAMPS
    if (item == 0 && tid == 0 && Q.stamps) Q.stamps[nl] = __builtin_amdgcn_s_memtime();   // start
#endif
    if (stage) {   // the observation -> buffer 1's region (layer 0's input), layer 0's parameters -> pwl
        const float4* src = reinterpret_cast<const float4*>(xg);
        float4* dst = reinterpret_cast<float4*>(buf[1]);
        for (int i = tid; i < D.in_feat / 4; i += DS_THREADS) dst[i] = src[i];
        for (int i = tid; i < D.L[0].pn; i += DS_THREADS) pwl[i] = flat[w0 + i];
    }
    for (int li = 0; li < nl; ++li) {
        const DsLayer L = D.L[li];
        __syncthreads();                                     // the layer's input and parameters in LDS
        if (li == 1 && stage) {
            // the staged observation is consumed: every conv's parameters into its
            // region (one batch of loads, one wait), then the barrier
            const float4* src = reinterpret_cast<const float4*>(flat + w0);
            float4* dst = reinterpret_cast<float4*>(pall);
            for (int i = tid; i < (D.ptot + 3) / 4; i += DS_THREADS) dst[i] = src[i];
            __syncthreads();
        }
        const ds_lptr lpw = (ds_lptr)(li == 0 ? pwl : pall + (L.woff - w0));
        const int Wi = L.Wi, Hi = L.Hi, Pi = Wi * Hi;
        const bool in_lds = L.in_buf >= 0 || stage;
        const ds_lptr inl = L.in_buf == 0 ? lb0 : lb1;       // (the staged observation sits at buffer 1)
        const ds_lptr outl = L.out_buf == 0 ? lb0 : lb1;
        const ds_lptr resl = L.res_buf == 0 ? lb0 : lb1;
        (void)Pi; (void)Hi;
        if (L.kind == DS_CONV) {
            // the 3x3 shapes of the configs[4] downsampler (4 -> 4 stride 2, 4 -> 4 on the VALU; 4 -> 8
            // stride 2, 8 -> 8 on MFMA; relu or identity), LDS to LDS; any other layer the generic way
            const bool k3 = stage && L.out_buf >= 0 && L.kw == 3 && L.kh == 3 && L.pw == 1 &&
                            L.ph == 1 && (L.act == MZ_ACT_RELU || L.act == MZ_ACT_IDENTITY);
            const int sel = !k3 ? -1
                          : L.cin == 4 && L.cout == 4 ? (L.stride == 2 ? 0 : L.stride == 1 ? 1 : -1)
                          : L.cin == 4 && L.cout == 8 && L.stride == 2 ? 2
                          : L.cin == 8 && L.cout == 8 && L.stride == 1 ? 3 : -1;
            if (sel == 0) ds_conv_valu<4, 4, 2>(L, inl, outl, resl, lpw, Q.bn_s);
            else if (sel == 1) ds_conv_valu<4, 4, 1>(L, inl, outl, resl, lpw, Q.bn_s);
            else if (sel == 2) ds_conv_mfma<4, 8, 2>(L, inl, outl, resl, lpw, Q.bn_s);
            else if (sel == 3) ds_conv_mfma<8, 8, 1>(L, inl, outl, resl, lpw, Q.bn_s);
            else {
                const float* in = L.in_buf < 0 ? (stage ? buf[1] : xg) : buf[L.in_buf];
                float* out = L.out_buf < 0 ? nullptr : buf[L.out_buf];
                const float* res = L.res_add ? buf[L.res_buf] : nullptr;
                ds_conv_generic(L, in, out, res, flat, Q.bn_s, yg, wl, kt, kd);
            }
        } else {
            ds_pool(L, inl, outl, yg);                       // (pools read an LDS buffer: never layer 0)
        }
        __syncthreads();
#ifdef MZ_STAMPS
        if (item == 0 && tid == 0 && Q.stamps) Q.stamps[li] = __builtin_amdgcn_s_memtime();
#endif
    }
}

// ---- the corrected learner through the downsampler (MZ_LEARN_CORRECTED on
// the configs[4] nets).  The same layers as mz_downsample_kernel, one
// workgroup per sample, every layer's output (and a BatchNorm conv's
// t = W x + b) kept in the sample's HBM arena for the backward and the
// parameter gradients.  Convs are gathers through Flux's flipped kernel with
// "same" padding and the layer's stride; MeanPool counts the padding.
__device__ __forceinline__ float dsbp_dz(int act, float g, float y) {
    return act == MZ_ACT_RELU ? (y > 0.0f ? g : 0.0f) : act == MZ_ACT_TANH ? g * (1.0f - y * y) : g;
}

extern "C" __global__ __launch_bounds__(DS_THREADS) void mz_dsbp_fwd(DsBpParams Q) {
    const DsPlan& D = *Q.plan;
    const int b = blockIdx.x, tid = threadIdx.x;
    float* T = Q.act + (size_t)b * Q.arena;
    const float* xg = Q.obs + (size_t)b * D.in_feat;
    for (int li = 0; li < D.n; ++li) {
        const DsLayer& L = D.L[li];
        const DsBpLayer A = Q.lay[li];
        const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Pi = Wi * Hi, Po = Wo * L.Ho;
        const float* in = A.x < 0 ? xg : T + A.x;
        const bool last = li == D.n - 1;
        for (int o = tid; o < L.cout * Po; o += DS_THREADS) {
            const int co = o / Po, p = o - co * Po, oh = p / Wo, ow = p - oh * Wo;
            float v;
            if (L.kind == DS_CONV) {
                const float* w = Q.flat + L.woff + (size_t)L.kw * L.kh * L.cin * co;
                float acc = 0.0f;
                for (int c = 0; c < L.cin; ++c)
                    for (int j = 0; j < L.kh; ++j) {
                        const int sy = L.stride * oh + (L.kh - 1 - j) - L.ph;
                        if (sy < 0 || sy >= Hi) continue;
                        for (int i = 0; i < L.kw; ++i) {
                            const int sx = L.stride * ow + (L.kw - 1 - i) - L.pw;
                            if (sx >= 0 && sx < Wi)
                                acc = __builtin_fmaf(w[i + L.kw * (j + L.kh * c)], in[sx + Wi * sy + Pi * c], acc);
                        }
                    }
                float t = acc + Q.flat[L.boff + co];
                if (L.bn) {
                    T[A.z + o] = t;
                    t = Q.flat[L.bnoff + L.cout + co] * ((t - 0.0f) / Q.bn_s) + Q.flat[L.bnoff + co];
                }
                if (L.res_add) t = t + T[A.res + o];
                v = L.act == MZ_ACT_RELU ? mz_relu(t) : L.act == MZ_ACT_TANH ? det_tanhf(t) : t;
            } else {
                float m = 0.0f;
                for (int j = 0; j < L.kh; ++j)
                    for (int i = 0; i < L.kw; ++i) {
                        const int sx = L.stride * ow + i - L.pw, sy = L.stride * oh + j - L.ph;
                        if (sx >= 0 && sx < Wi && sy >= 0 && sy < Hi) m = m + in[sx + Wi * sy + Pi * co];
                    }
                v = (1.0f / (float)(L.kw * L.kh)) * m;
            }
            T[A.y + o] = v;
            if (last) Q.out[(size_t)b * D.out_feat + o] = v;
        }
        __syncthreads();
    }
}

// Input gradients, layers in reverse: a conv's ∂L/∂t (into dt_off) after its
// relu' (the residual input receives ∂L/∂u unchanged) and BatchNorm's
// γ/√(1+ε); then ∂L/∂x, one thread per input element gathering over the output
// channels and the taps that read it (the transposed strided conv); a
// MeanPool spreads ∂L/∂y over its windows.  Accumulation into a tensor's
// ∂L/∂x happens in the layers' reverse order, one layer per barrier.
extern "C" __global__ __launch_bounds__(DS_THREADS) void mz_dsbp_bwd(DsBpParams Q) {
    const DsPlan& D = *Q.plan;
    const int b = blockIdx.x, tid = threadIdx.x;
    const float* T = Q.act + (size_t)b * Q.arena;
    float* G = Q.grad + (size_t)b * Q.arena;
    float* DT = G + Q.dt_off;
    for (int e = tid; e < Q.dt_off; e += DS_THREADS) G[e] = 0.0f;
    __syncthreads();
    {
        const DsBpLayer A = Q.lay[D.n - 1];
        for (int f = tid; f < D.out_feat; f += DS_THREADS) G[A.y + f] = Q.gout[(size_t)b * Q.gstride + Q.goff + f];
    }
    __syncthreads();
    for (int li = D.n - 1; li >= 0; --li) {
        const DsLayer& L = D.L[li];
        const DsBpLayer A = Q.lay[li];
        const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Ho = L.Ho, Pi = Wi * Hi, Po = Wo * Ho;
        if (L.kind == DS_CONV) {
            for (int o = tid; o < L.cout * Po; o += DS_THREADS) {
                const int co = o / Po;
                const float du = dsbp_dz(L.act, G[A.y + o], T[A.y + o]);
                if (L.res_add) G[A.res + o] += du;
                DT[o] = L.bn ? du * (Q.flat[L.bnoff + L.cout + co] / Q.bn_s) : du;
            }
            __syncthreads();
        }
        if (A.x >= 0) {
            const float* dy = L.kind == DS_CONV ? DT : G + A.y;
            const int K = L.kw * L.kh * L.cin;
            for (int e = tid; e < L.cin * Pi; e += DS_THREADS) {
                const int c = e / Pi, q = e - c * Pi, sy = q / Wi, sx = q - sy * Wi;
                float acc = 0.0f;
                if (L.kind == DS_CONV) {
                    for (int co = 0; co < L.cout; ++co) {
                        const float* w = Q.flat + L.woff + (size_t)K * co + (size_t)L.kw * L.kh * c;
                        for (int j = 0; j < L.kh; ++j) {
                            const int ny = sy - (L.kh - 1 - j) + L.ph;
                            if (ny < 0 || ny % L.stride) continue;
                            const int oh = ny / L.stride;
                            if (oh >= Ho) continue;
                            for (int i = 0; i < L.kw; ++i) {
                                const int nx = sx - (L.kw - 1 - i) + L.pw;
                                if (nx < 0 || nx % L.stride) continue;
                                const int ow = nx / L.stride;
                                if (ow < Wo) acc = __builtin_fmaf(w[i + L.kw * j], dy[co * Po + oh * Wo + ow], acc);
                            }
                        }
                    }
                } else {
                    for (int j = 0; j < L.kh; ++j) {
                        const int ny = sy - j + L.ph;
                        if (ny < 0 || ny % L.stride) continue;
                        const int oh = ny / L.stride;
                        if (oh >= Ho) continue;
                        for (int i = 0; i < L.kw; ++i) {
                            const int nx = sx - i + L.pw;
                            if (nx < 0 || nx % L.stride) continue;
                            const int ow = nx / L.stride;
                            if (ow < Wo) acc += dy[c * Po + oh * Wo + ow];
                        }
                    }
                    acc = (1.0f / (float)(L.kw * L.kh)) * acc;
                }
                G[A.x + e] += acc;
            }
        }
        __syncthreads();
    }
}

// Parameter gradients: one workgroup per (conv, output channel co, input
// channel ci).  Thread (k, s) sums column k of the pair's im2col product
// (k < kw·kh: the tap's W; with ci = 0 also db, dβ, dγ) over the (sample,
// position) pairs s, s + S, ..; the S partial sums are added in ascending s.
// Also the Σθ² of the job's parameters.
extern "C" __global__ __launch_bounds__(DS_DW_THREADS) void mz_dsbp_dw(DsDwParams Q) {
    __shared__ float red[DS_DW_THREADS];
    const DsPlan& D = *Q.plan;
    const DsDwJob J = Q.jobs[blockIdx.x];
    const DsLayer& L = D.L[J.layer];
    const DsBpLayer A = Q.lay[J.layer];
    const int tid = threadIdx.x, co = J.co, c = J.ci;
    const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Pi = Wi * Hi, Po = Wo * L.Ho;
    const int kk = L.kw * L.kh, K = kk * L.cin, nk = kk + (c == 0 ? (L.bn ? 3 : 1) : 0), S = DS_DW_THREADS / nk;
    const int k = tid % nk, s = tid / nk;
    const float gr = L.bn ? Q.flat[L.bnoff + L.cout + co] / Q.bn_s : 1.0f;
    int dx = 0, dy = 0;
    if (k < kk) {
        const int j = k / L.kw, i = k - j * L.kw;
        dx = (L.kw - 1 - i) - L.pw; dy = (L.kh - 1 - j) - L.ph;
    }
    float acc = 0.0f;
    if (s < S) {
        for (int pr = s; pr < Q.B * Po; pr += S) {
            const int b = pr / Po, p = pr - b * Po, oh = p / Wo, ow = p - oh * Wo;
            const float* T = Q.act + (size_t)b * Q.arena;
            const float* G = Q.grad + (size_t)b * Q.arena;
            const int e = co * Po + p;
            const float du = dsbp_dz(L.act, G[A.y + e], T[A.y + e]);
            if (k < kk) {
                const int sx = L.stride * ow + dx, sy = L.stride * oh + dy;
                const float* X = A.x < 0 ? Q.obs + (size_t)b * D.in_feat : T + A.x;
                const float xv = sx >= 0 && sx < Wi && sy >= 0 && sy < Hi ? X[sx + Wi * sy + Pi * c] : 0.0f;
                acc = __builtin_fmaf(du * gr, xv, acc);
            } else if (k == kk) {
                acc += du * gr;
            } else if (k == kk + 1) {
                acc += du;
            } else {
                acc += du * (T[A.z + e] / Q.bn_s);
            }
        }
    }
    red[tid] = acc;
    __syncthreads();
    const size_t w0 = (size_t)L.woff + (size_t)K * co + (size_t)kk * c;
    if (tid < nk) {
        float t = 0.0f;
        for (int r = 0; r < S; ++r) t += red[tid + r * nk];
        const size_t dst = tid < kk ? w0 + tid
                         : tid == kk ? (size_t)L.boff + co
                         : tid == kk + 1 ? (size_t)L.bnoff + co : (size_t)L.bnoff + L.cout + co;
        Q.out[dst] = t;
    }
    if (tid == 0) {
        double q = 0.0;
        for (int i = 0; i < kk; ++i) { const double w = Q.flat[w0 + i]; q += w * w; }
        if (c == 0) {
            const double bb = Q.flat[L.boff + co];
            q += bb * bb;
            if (L.bn) {
                const double be = Q.flat[L.bnoff + co], ga = Q.flat[L.bnoff + L.cout + co];
                q += be * be + ga * ga;
            }
        }
        Q.sq[blockIdx.x] = q;
    }
}
