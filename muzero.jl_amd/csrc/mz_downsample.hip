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
