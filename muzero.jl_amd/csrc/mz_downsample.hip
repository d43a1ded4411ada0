// mz_downsample.hip — the downsampler of the ResNet representation
// (ResNetHP.downsample, src/Learning.jl:175-187) for BASELINE configs[4]
// (84x84x4 observations): one workgroup per item runs every layer of the
// DsPlan with the activations in LDS; the result (6, 6, 2C) goes to HBM,
// where the representation's tail (mz_rsearch_root / mz_runroll_kernel /
// mz_rnet_forward_kernel) reads it as its input.
//
// Numerics = oracle/mz_oracle.c conv_fwd / pool_fwd bit for bit: each output
// is the canonical dot (four k-quarter fmaf chains of length 4⌈K/16⌉ over
// k = i + kw·j + kw·kh·c, ((p0+p1)+(p2+p3))) + bias, then BatchNorm
// γ·((t - 0)/s) + β, the block input, the activation; MeanPool sums the
// in-board window rows outer / columns inner and multiplies by f32(1/9).
// The work is small (≈ 3.3 M MACs per item, once per move) next to the
// S simulations of the search, so it runs on the VALU with LDS-staged
// weights (wave-uniform output channel: broadcast reads).
#include <hip/hip_runtime.h>
#include "mz_internal.h"
#include "mz_resnet_params.h"

__device__ __forceinline__ float ds_act(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

extern "C" __global__ __launch_bounds__(DS_THREADS) void mz_downsample_kernel(DsParams Q) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const DsPlan& D = *Q.plan;
    const int item = blockIdx.x, tid = threadIdx.x;
    float* buf[2] = {lds, lds + D.buf_floats};
    float* wl = lds + 2 * D.buf_floats;                      // [cout][K] weights of the current conv
    int* kt = reinterpret_cast<int*>(wl + D.w_floats);       // [K]: c·Pi + dy·Wi + dx
    int* kd = kt + 256;                                      // [K]: (dx + 8) | (dy + 8) << 4
    const float* xg = Q.x + (size_t)item * D.in_feat;
    for (int li = 0; li < D.n; ++li) {
        const DsLayer& L = D.L[li];
        const int Wi = L.Wi, Hi = L.Hi, Wo = L.Wo, Ho = L.Ho, Pi = Wi * Hi, Po = Wo * Ho;
        const float* in = L.in_buf < 0 ? xg : buf[L.in_buf];
        float* out = L.out_buf < 0 ? nullptr : buf[L.out_buf];
        const float* res = L.res_add ? buf[L.res_buf] : nullptr;
        if (L.kind == DS_CONV) {
            const int K = L.kw * L.kh * L.cin;
            for (int i = tid; i < K * L.cout; i += DS_THREADS) wl[i] = Q.flat[L.woff + i];
            for (int k = tid; k < K; k += DS_THREADS) {
                const int i = k % L.kw, j = (k / L.kw) % L.kh, c = k / (L.kw * L.kh);
                const int dx = (L.kw - 1 - i) - L.pw, dy = (L.kh - 1 - j) - L.ph;   // Flux: kernel flipped
                kt[k] = c * Pi + dy * Wi + dx;
                kd[k] = (dx + 8) | ((dy + 8) << 4);
            }
            __syncthreads();
            const int kq = 4 * ((K + 15) / 16);
            for (int o = tid; o < L.cout * Po; o += DS_THREADS) {
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
                float t = ((part[0] + part[1]) + (part[2] + part[3])) + Q.flat[L.boff + co];
                if (L.bn) t = Q.flat[L.bnoff + L.cout + co] * ((t - 0.0f) / Q.bn_s) + Q.flat[L.bnoff + co];
                if (res) t = t + res[o];
                t = ds_act(L.act, t);
                if (out) out[o] = t;
                else Q.y[(size_t)item * D.out_feat + o] = t;
            }
        } else {                                            // MeanPool (no flip), padding counted
            const float inv = 1.0f / (float)(L.kw * L.kh);
            for (int o = tid; o < L.cout * Po; o += DS_THREADS) {
                const int c = o / Po, p = o - c * Po;
                const int oh = p / Wo, ow = p - oh * Wo;
                float m = 0.0f;
                for (int j = 0; j < L.kh; ++j)
                    for (int i = 0; i < L.kw; ++i) {
                        const int sx = L.stride * ow + i - L.pw, sy = L.stride * oh + j - L.ph;
                        if (sx >= 0 && sx < Wi && sy >= 0 && sy < Hi) m = m + in[sx + Wi * sy + Pi * c];
                    }
                const float t = inv * m;
                if (out) out[o] = t;
                else Q.y[(size_t)item * D.out_feat + o] = t;
            }
        }
        __syncthreads();
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
