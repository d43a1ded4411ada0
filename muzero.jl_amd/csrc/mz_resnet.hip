// mz_resnet.hip — the ResNet networks (row a14; Learning.jl:148-255, the
// intended architecture of SURVEY §2.1 Q12) on f32 MFMA, one tile of NG games
// per RN_THREADS-thread workgroup, activations resident in LDS across all layers.
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
#include "mz_replay_device.h"

__device__ __forceinline__ float rn_act(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

// A fragments of 16 output rows (block ob) for chunk c = k-steps 4c..4c+3 of
// the four quarter chains: a[q][jj] (image [ob][q][nq4/4][lane][4]).
__device__ __forceinline__ void rn_load_a(float (*a)[4], const float* __restrict__ Wimg, const RLayer& L,
                                          int ob, int c, int lane) {
    const int nch = (L.nq + 3) >> 2;
    #ifdef RN_HOTA
    const float* base = Wimg + (size_t)ob
#else
    const float* base = Wimg + L.w_img + (size_t)ob
#endif
                       * (16 * nch * 64) + (size_t)lane * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(base + (size_t)((q * nch + c) * 64) * 4);
        a[q][0] = v.x; a[q][1] = v.y; a[q][2] = v.z; a[q][3] = v.w;
    }
}

// Epilogue of NB 16x16 accumulator sets (column blocks of one lane: n[i],
// row block ob): ((p0+p1)+(p2+p3)) + b, BatchNorm in test mode, residual,
// activation -> out[o][n].  The BatchNorm quotient (t − 0)/s uses r = 1/s:
// q0 = t·r, e = fma(−q0, s, t), q0 + e·r is the IEEE quotient for every
// finite float with |t| >= 2^-100 (exhaustive check: tools/check_bn_div.c,
// tests/test_bn_div.py); below that, where e underflows, and for ±inf / NaN
// (q0 = ±inf makes e NaN, where IEEE gives ±inf: hidden states overflow once
// Q1's in-place doubling has run ~128 levels deep, configs[4]), one
// wave-uniform branch divides.
// bias, γ, β of the 4 rows a lane holds in row block ob (issued before the
// MFMAs of the unit so their latency hides under them)
// (from the layer's epilogue image: four 16-byte loads; rows past cout and the
// BatchNorm entries of layers without one read 0)
__device__ __forceinline__ void rn_load_ep(float (&ep)[3][4], const RLayer& L, const float* __restrict__ Wimg,
                                           int ob, int kl) {
    #ifdef RN_HOTA
    const float4* e = reinterpret_cast<const float4*>(Wimg) + ob * 16 + kl * 4;
#else
    const float4* e = reinterpret_cast<const float4*>(Wimg + L.ep_img) + ob * 16 + kl * 4;
#endif
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float4 v = e[r];
        ep[0][r] = v.x; ep[1][r] = v.y; ep[2][r] = v.z;
    }
}
// A layer's packed entry by scalar load (constant address space: the plans
// are never written by the kernels)
__device__ __forceinline__ RLayer rn_layer_at(const RPlan& R, int i) {
#ifdef __HIP_DEVICE_COMPILE__
    typedef const __attribute__((address_space(4))) int4* cp4;
    const cp4 k = (cp4)(&R.k[0]);
    const int4 a = k[2 * i], b = k[2 * i + 1];
    const RK x = {{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
    return rn_rk_decode(x);
#else
    return rn_rk_decode(R.k[i]);
#endif
}

// LDS index of output row o = ob·16 + kl·4 + r, column n, in layout kb
__device__ __forceinline__ int rn_out_idx(int kb, int ob, int kl, int r, int n, int ncols) {
    return kb ? (ob * ncols + n) * 16 + 4 * (((n >> 2) & 3) ^ rn_kb_sigma(r)) + kl   // rn_kb_off(o, n)
              : (ob * 16 + kl * 4 + r) * ncols + n;
}
// the residual operands of a unit, read before its MFMAs (their LDS latency
// then hides under the chunks); 0 for rows / columns past the layer
template <int NB>
__device__ __forceinline__ void rn_load_res(const RLayer& L, const float* lds, float (&res)[NB][4], int ob, int kl,
                                            const int (&n)[NB], int ncols) {
    if (!L.res_add) {                                   // wave-uniform
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) res[i][r] = 0.0f;
        return;
    }
    // branch-free: out-of-tile lanes read a clamped in-range element, then take 0
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const bool in = ob * 16 + kl * 4 + r < L.cout && n[i] < ncols;
            const int nc = n[i] < ncols ? n[i] : ncols - 1;
            const int oc = ob * 16 + kl * 4 + r < L.cout ? ob : 0;
            const float x = lds[L.res_off + rn_out_idx(L.res_kb, oc, kl, ob * 16 + kl * 4 + r < L.cout ? r : 0, nc,
                                                       ncols)];
            res[i][r] = in ? x : 0.0f;
        }
}

// The common case of rn_epilogue, the same operations without per-element
// branches: a full 16-row block (o < cout for all rows) and a relu / identity
// activation; the layout, BatchNorm and residual choices are wave-uniform and
// taken once, outside the element loops (OUT_KB, RES, RELU instances).
template <int NB, bool OUT_KB, bool RES, bool RELU>
__device__ __forceinline__ void rn_epilogue_full(const RLayer& L, const float (&d)[NB][4], float* lds, int ob, int kl,
                                                 const int (&n)[NB], int ncols, const float (&res)[NB][4]) {
    float* out = lds + L.out_off;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = d[i][r];
            if constexpr (RES) v[r] = v[r] + res[i][r];
            if constexpr (RELU) v[r] = mz_relu(v[r]);
        }
        if (n[i] < ncols) {
#pragma unroll
            for (int r = 0; r < 4; ++r) out[rn_out_idx(OUT_KB, ob, kl, r, n[i], ncols)] = v[r];
        }
    }
}

template <int NB, bool RAWTANH = false>
__device__ __forceinline__ void rn_epilogue(const RLayer& L, const mz_f32x4 (&acc)[NB][4], const float (&ep)[3][4],
                                            float* lds, int ob, int kl, const int (&n)[NB], int ncols, float bn_s,
                                            float bn_r, const float (&res)[NB][4]) {
    float d[NB][4];
    bool tiny = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float bias = ep[0][r];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            float t = (acc[i][0][r] + acc[i][1][r]) + (acc[i][2][r] + acc[i][3][r]);
            t = t + bias;
            d[i][r] = t;
            tiny |= !(fabsf(t) >= 0x1p-100f) || fabsf(t) == INFINITY;   // tiny, ±inf or NaN
        }
    }
    if (L.bn) {
        float q[NB][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const float t = d[i][r] - 0.0f;
                const float q0 = t * bn_r;
                const float e = fmaf(-q0, bn_s, t);
                q[i][r] = fmaf(e, bn_r, q0);
            }
        if (__builtin_expect(__ballot(tiny) != 0, 0)) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < NB; ++i)
                    if (!(fabsf(d[i][r]) >= 0x1p-100f) || fabsf(d[i][r]) == INFINITY)
                        q[i][r] = (d[i][r] - 0.0f) / bn_s;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < NB; ++i) d[i][r] = ep[1][r] * q[i][r] + ep[2][r];
    }
    if ((ob + 1) * 16 <= L.cout && L.act != MZ_ACT_TANH) {
        const bool relu = L.act == MZ_ACT_RELU;
#define RN_EF(KB, RS, RL) rn_epilogue_full<NB, KB, RS, RL>(L, d, lds, ob, kl, n, ncols, res)
        if (L.out_kb) {
            if (L.res_add) { if (relu) RN_EF(true, true, true); else RN_EF(true, true, false); }
            else { if (relu) RN_EF(true, false, true); else RN_EF(true, false, false); }
        } else {
            if (L.res_add) { if (relu) RN_EF(false, true, true); else RN_EF(false, true, false); }
            else { if (relu) RN_EF(false, false, true); else RN_EF(false, false, false); }
        }
#undef RN_EF
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int o = ob * 16 + kl * 4 + r;
        if (o >= L.cout) continue;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            if (n[i] >= ncols) continue;
            float v = d[i][r];
            if (L.res_add) v = v + res[i][r];
            // RAWTANH: no det_tanhf (f64) code in the layer loop; the read-out applies it
            lds[L.out_off + rn_out_idx(L.out_kb, ob, kl, r, n[i], ncols)] =
                RAWTANH ? (L.act == MZ_ACT_RELU ? mz_relu(v) : v) : rn_act(L.act, v);
        }
    }
}

// One layer, barrier-separated from its neighbours (Dense layers, kernels
// > 1x1).  A wave owns a unit = one 16-row output block x NBW 16-column
// blocks; each A fragment feeds NBW MFMAs and the four k-quarter chains of
// every 16x16 tile run as four accumulators (canonical order: chain q takes
// k = (q·NQ + j)·4 + (lane>>4) for j ascending).  The wave walks (unit, chunk
// of 4 k-steps) pairs, the A fragments of the next pair loaded before the
// MFMAs of the current one; a chunk's B operands are read from LDS in one
// batch.  B(k, n): MODE 0 Dense / MODE 1 1x1 conv read x[k][n]; MODE 2
// (kernel > 1x1) reads
// through the k table: t = off·256 | (dx+8)·16 | (dy+8) with off = ch·ncols +
// (dx + W·dy)·NG, zero outside the board.  Addresses are clamped in range and
// out-of-range operands selected to 0 (no branches).
// Operands of a wave's first unit of a layer, loaded before the barrier that
// ends the previous layer (rn_run<.., PF = true>): its first chunk of A
// fragments and its epilogue parameters.  Without this every layer starts
// with a dependent round trip to L2 for the plan, then one for the weights.
struct RnPf {
    float an[4][4];
    float ep[3][4];
};

template <int NBW, int MODE, bool PF = false, bool PIPE = false, bool RAWTANH = false>
__device__ __forceinline__ void rn_layer_t(const RLayer& L, const float* __restrict__ Wimg,
                                           const float* __restrict__ flat, float* lds, int NG, int Wb, int P,
                                           float bn_s, float bn_r, const RnPf* pf = nullptr,
                                           unsigned long long* dbg = nullptr) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwaves = blockDim.x >> 6;
#ifdef MZ_STAMPS   // diagnostic build: phases of wave 0's first unit (waits forced, so approximate)
#define RN_DBG(k)                                                                                     \
    do {                                                                                              \
        if (dbg && threadIdx.x == 0 && u == 0) dbg[k] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#define RN_DBG_WAIT(k)                                                                                \
    do {                                                                                              \
        if (dbg && u == 0) { __builtin_amdgcn_s_waitcnt(0); RN_DBG(k); }                              \
    } while (0)
#else
#define RN_DBG(k) do {} while (0)
#define RN_DBG_WAIT(k) do {} while (0)
#endif
    (void)dbg;
    // MODE 3: a 1x1 conv / Dense reading a k-blocked input (K % 64 == 0)
    const int ncols = MODE == 0 ? NG : MODE == 3 ? (L.spatial ? P * NG : NG) : P * NG;
    const int n_nb = (ncols + 15) >> 4;
    const int n_grp = (n_nb + NBW - 1) / NBW;
    const int units = L.n_ob * n_grp;
    const int NQ = L.nq, K = L.K, Hb = P / Wb, nch = (NQ + 3) >> 2;
    const int kl = lane >> 4;
    const int* tab = reinterpret_cast<const int*>(lds) + L.ktab;
    int u = wave;
    if (u >= units) return;
    RN_DBG(0);
    float an[4][4];
    if constexpr (PF) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) an[q][jj] = pf->an[q][jj];
    } else {
        rn_load_a(an, Wimg, L, u / n_grp, 0, lane);
    }
    for (; u < units; u += nwaves) {
        const int ob = u / n_grp, grp = u - ob * n_grp;
        float ep[3][4];
        if (PF && u == wave) {
#pragma unroll
            for (int e = 0; e < 3; ++e)
#pragma unroll
                for (int r = 0; r < 4; ++r) ep[e][r] = pf->ep[e][r];
        } else {
            rn_load_ep(ep, L, Wimg, ob, kl);
        }
        int cb[NBW], cw[NBW], chh[NBW];
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
            const int n = (grp * NBW + i) * 16 + (lane & 15);
            const int nn = n < ncols ? n : ncols - 1;
            cb[i] = L.in_off + nn;
            if (MODE == 2) {
                const int pp = nn / NG;
                cw[i] = pp % Wb; chh[i] = pp / Wb;
            }
        }
        // MODE 0/1: byte address of row q·NQ·4 + kl at each column block; the
        // k-step adds a wave-uniform j·4·ncols; kq[q] = rows of quarter q left
        // for this lane (k < K)
        // MODE 3: byte address of this lane's 16-byte piece of chunk 0 of quarter
        // q (the four k-steps (q·NQ + 4c + jj)·4 + kl, jj = 0..3; chunk c adds
        // a wave-uniform c·ncols·64 bytes)
        uint32_t bq[4][NBW];
        int kq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            kq[q] = K - (q * NQ * 4 + kl);
#pragma unroll
            for (int i = 0; i < NBW; ++i) bq[q][i] = (uint32_t)(cb[i] + (q * NQ * 4 + kl) * ncols) * 4u;
        }
        mz_f32x4 acc[NBW][4];
#pragma unroll
        for (int i = 0; i < NBW; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[i][q] = mz_f32x4{0.f, 0.f, 0.f, 0.f};
        int nn[NBW];
#pragma unroll
        for (int i = 0; i < NBW; ++i) nn[i] = (grp * NBW + i) * 16 + (lane & 15);
        // one-column-block units (the learner chain's) read their residual
        // operands up front; wider units in the epilogue (register budget of the
        // 12-wave network kernel)
        float res[NBW][4];
        if constexpr (NBW == 1) rn_load_res<NBW>(L, lds, res, ob, kl, nn, ncols);
        RN_DBG_WAIT(1);                                 // operands of the first chunk in registers
        if constexpr (MODE == 4) {
            // offset table (narrow plans): per quarter one 16-byte read of the
            // chunk's four B addresses, then the four B reads; no address VALU
            const int nch4 = ((NQ + 3) & ~3) / 4, ncols_t = n_grp * NBW * 16;
            const int n0 = grp * NBW * 16 + (lane & 15);
            const int* tb = reinterpret_cast<const int*>(lds) + L.ktab + n0 * 16 +
                            4 * (((n0 >> 2) & 3) ^ rn_kb_sigma(kl));
            constexpr int QG = NBW == 1 ? 4 : 2;
            if constexpr (PIPE && NBW == 1) {
                // software-pipelined (the 256-thread chain kernel's register room):
                // chunk c's MFMAs run under the B reads of chunk c + 1 and the
                // offset reads of chunk c + 2 (past the end: re-reads, unused)
                const char* lb = reinterpret_cast<const char*>(lds);
                auto rd_o = [&](int c, int4 (&o)[4]) {
#pragma unroll
                    for (int h = 0; h < 4; ++h) o[h] = *reinterpret_cast<const int4*>(tb + (h * nch4 + c) * ncols_t * 16);
                };
                auto rd_b = [&](const int4 (&o)[4], float (&bv)[4][4]) {
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        bv[h][0] = *reinterpret_cast<const float*>(lb + o[h].x);
                        bv[h][1] = *reinterpret_cast<const float*>(lb + o[h].y);
                        bv[h][2] = *reinterpret_cast<const float*>(lb + o[h].z);
                        bv[h][3] = *reinterpret_cast<const float*>(lb + o[h].w);
                    }
                };
                int4 o1[4];
                float bv[4][4];
                rd_o(0, o1);
                rd_b(o1, bv);
                rd_o(nch4 > 1 ? 1 : 0, o1);
                for (int c = 0; c < nch4; ++c) {
                    float ac[4][4];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) ac[q][jj] = an[q][jj];
                    {
                        const int un = c + 1 < nch4 ? u : u + nwaves, cn = c + 1 < nch4 ? c + 1 : 0;
                        if (un < units) rn_load_a(an, Wimg, L, un / n_grp, cn, lane);
                    }
                    float bn[4][4];
                    int4 o2[4];
                    rd_b(o1, bn);
                    rd_o(c + 2 < nch4 ? c + 2 : nch4 - 1, o2);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            acc[0][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[q][jj], bv[q][jj], acc[0][q], 0, 0, 0);
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        o1[h] = o2[h];
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) bv[h][jj] = bn[h][jj];
                    }
                }
            } else
            for (int c = 0; c < nch4; ++c) {
                float ac[4][4];                         // this chunk's A; the next one's loads fly under it
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) ac[q][jj] = an[q][jj];
                {
                    const int un = c + 1 < nch4 ? u : u + nwaves, cn = c + 1 < nch4 ? c + 1 : 0;
                    if (un < units) rn_load_a(an, Wimg, L, un / n_grp, cn, lane);
                }
#pragma unroll
                for (int qp = 0; qp < 4; qp += QG) {
                    int4 o[QG][NBW];
#pragma unroll
                    for (int h = 0; h < QG; ++h)
#pragma unroll
                        for (int i = 0; i < NBW; ++i)
                            o[h][i] = *reinterpret_cast<const int4*>(tb + ((qp + h) * nch4 + c) * ncols_t * 16 + 256 * i);
                    float bv[QG][NBW][4];
#pragma unroll
                    for (int h = 0; h < QG; ++h)
#pragma unroll
                        for (int i = 0; i < NBW; ++i) {
                            const char* lb = reinterpret_cast<const char*>(lds);
                            bv[h][i][0] = *reinterpret_cast<const float*>(lb + o[h][i].x);
                            bv[h][i][1] = *reinterpret_cast<const float*>(lb + o[h][i].y);
                            bv[h][i][2] = *reinterpret_cast<const float*>(lb + o[h][i].z);
                            bv[h][i][3] = *reinterpret_cast<const float*>(lb + o[h][i].w);
                        }
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                        for (int h = 0; h < QG; ++h)
#pragma unroll
                            for (int i = 0; i < NBW; ++i)
                                acc[i][qp + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[qp + h][jj], bv[h][i][jj],
                                                                                      acc[i][qp + h], 0, 0, 0);
                }
            }
        } else if constexpr (MODE == 3) {
            // k-blocked input: per quarter one 16-byte LDS read per column block
            // (unclamped columns: past-the-tile lanes read spare LDS, their
            // results are discarded); A used in place, the next chunk's fetched
            // after this chunk's MFMAs (1x1 convs over 64 channels have one)
            const int n0 = grp * NBW * 16 + (lane & 15);
            const uint32_t b0 = (uint32_t)(L.in_off + n0 * 16 + 4 * (((n0 >> 2) & 3) ^ rn_kb_sigma(kl))) * 4u;
            for (int c = 0; c < nch; ++c) {
                constexpr int QG = NBW == 1 ? 4 : 2;
#pragma unroll
                for (int qp = 0; qp < 4; qp += QG) {
                    float4 v[QG][NBW];
#pragma unroll
                    for (int h = 0; h < QG; ++h) {
                        const char* base = reinterpret_cast<const char*>(lds) + b0 +
                                           (uint32_t)(((qp + h) * NQ / 4 + c) * ncols) * 64u;
#pragma unroll
                        for (int i = 0; i < NBW; ++i) v[h][i] = *reinterpret_cast<const float4*>(base + 1024 * i);
                    }
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                        for (int h = 0; h < QG; ++h)
#pragma unroll
                            for (int i = 0; i < NBW; ++i) {
                                const float bv = jj == 0 ? v[h][i].x : jj == 1 ? v[h][i].y : jj == 2 ? v[h][i].z
                                                                                                    : v[h][i].w;
                                acc[i][qp + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(an[qp + h][jj], bv,
                                                                                      acc[i][qp + h], 0, 0, 0);
                            }
                }
                const int un = c + 1 < nch ? u : u + nwaves, cn = c + 1 < nch ? c + 1 : 0;
                if (un < units) rn_load_a(an, Wimg, L, un / n_grp, cn, lane);
            }
        } else
        for (int c = 0; c < nch; ++c) {
            float ac[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) ac[q][jj] = an[q][jj];
            {                                           // prefetch the next (unit, chunk) or layer
                const int un = c + 1 < nch ? u : u + nwaves, cn = c + 1 < nch ? c + 1 : 0;
                if (un < units) rn_load_a(an, Wimg, L, un / n_grp, cn, lane);
            }
            float b[4][4][NBW];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = (q * NQ + 4 * c + jj) * 4 + kl;
                    const bool kin = k < K && 4 * c + jj < NQ;
                    const int kc = kin ? k : K - 1;
                    if (MODE == 2) {
                        const int t = tab[kc];
                        const int off = t >> 8, dx = ((t >> 4) & 15) - 8, dy = (t & 15) - 8;
#pragma unroll
                        for (int i = 0; i < NBW; ++i) {
                            const bool ok = kin && (unsigned)(cw[i] + dx) < (unsigned)Wb &&
                                            (unsigned)(chh[i] + dy) < (unsigned)Hb;
                            const float v = lds[ok ? cb[i] + off : cb[i]];
                            b[jj][q][i] = ok ? v : 0.0f;
                        }
                    } else {
                        const uint32_t so = (uint32_t)((4 * c + jj) * 4 * ncols) * 4u;
                        const bool kv = 4 * (4 * c + jj) < kq[q];
#pragma unroll
                        for (int i = 0; i < NBW; ++i) {
                            const float v = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(lds) +
                                                                            bq[q][i] + so);
                            b[jj][q][i] = kv ? v : 0.0f;
                        }
                    }
                }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                if (4 * c + jj >= NQ) break;
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < NBW; ++i)
                        acc[i][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[q][jj], b[jj][q][i], acc[i][q], 0, 0, 0);
            }
        }
#ifdef MZ_STAMPS
        if (dbg && u == 0) {
#pragma unroll
            for (int i = 0; i < NBW; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) asm volatile("s_nop 7" :: "v"(acc[i][q]));
        }
#endif
        RN_DBG_WAIT(2);                                 // chunks done (MFMA results consumed)
        if constexpr (NBW != 1) rn_load_res<NBW>(L, lds, res, ob, kl, nn, ncols);
        rn_epilogue<NBW, RAWTANH>(L, acc, ep, lds, ob, kl, nn, ncols, bn_s, bn_r, res);
        RN_DBG_WAIT(3);                                 // epilogue stored
    }
}

#ifndef RN_NBW
#define RN_NBW 3
#endif
// Column blocks per unit of layer L (the rn_layer_t instance rn_layer picks):
// narrow tiles (the learner chain's, a few items on a small board) have fewer
// than 3 column blocks, so a unit of exactly that many (no MFMAs on columns
// past the tile)
template <bool NARROW>
__device__ __forceinline__ int rn_nbw(const RLayer& L, int NG, int P) {
    if (!L.spatial) return 1;
    const int n_nb = NARROW ? (P * NG + 15) >> 4 : 3;
    return n_nb == 1 ? 1 : n_nb == 2 ? 2 : L.kk > 1 ? 3 : RN_NBW;
}

// NBWMAX = 1: a narrow kernel instance for tiles of one column block (the host
// launches it only then): the 1-block units alone, a fifth of the code
template <bool NARROW, bool PF = false, int NBWMAX = 3, bool PIPE = false, bool NOKK = false, bool RAWTANH = false>
__device__ __forceinline__ void rn_layer(const RLayer& L, const float* __restrict__ Wimg,
                                         const float* __restrict__ flat, float* lds, int NG, int Wb, int P,
                                         float bn_s, float bn_r, const RnPf* pf = nullptr,
                                         unsigned long long* dbg = nullptr) {
    const int n_nb = NBWMAX == 1 ? 1 : NARROW && L.spatial ? (P * NG + 15) >> 4 : 3;     // as rn_nbw
#define RN_L(NB, M) rn_layer_t<NB, M, PF, PIPE, RAWTANH>(L, Wimg, flat, lds, NG, Wb, P, bn_s, bn_r, pf, dbg)
    if (NARROW && L.otab) {                                           // kernel > 1x1 through the offset table
        if (n_nb == 1) RN_L(1, 4);
        else if constexpr (NBWMAX > 1) { if (n_nb == 2) RN_L(2, 4); else RN_L(3, 4); }
    } else if (L.in_kb) {                                             // 1x1 conv / Dense, K % 64 == 0
        if (!L.spatial || n_nb == 1) RN_L(1, 3);
        else if constexpr (NBWMAX > 1) { if (n_nb == 2) RN_L(2, 3); else RN_L(RN_NBW, 3); }
    } else if (!NOKK && L.kk > 1) {              // (NOKK: plans of 1x1 convs and Dense layers only)
        if constexpr (!NOKK) {
            if (n_nb == 1) RN_L(1, 2);
            else if constexpr (NBWMAX > 1) { if (n_nb == 2) RN_L(2, 2); else RN_L(3, 2); }
        }
    } else if (L.spatial) {
        if (n_nb == 1) RN_L(1, 1);
        else if constexpr (NBWMAX > 1) { if (n_nb == 2) RN_L(2, 1); else RN_L(RN_NBW, 1); }
    } else {
        RN_L(1, 0);
    }
#undef RN_L
}

// This wave's first-unit operands of layer L (no-op for a wave without one)
template <bool NARROW, int NBWMAX = 3>
__device__ __forceinline__ void rn_prefetch(const RLayer& L, const float* __restrict__ Wimg,
                                            const float* __restrict__ flat, int NG, int P, RnPf& pf) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ncols = L.spatial ? P * NG : NG;
    const int nbw = NBWMAX == 1 ? 1 : rn_nbw<NARROW>(L, NG, P);      // (rn_layer's unit width)
    const int n_grp = (((ncols + 15) >> 4) + nbw - 1) / nbw;
    if (wave < L.n_ob * n_grp) {
        const int ob = wave / n_grp;
        rn_load_a(pf.an, Wimg, L, ob, 0, lane);
        rn_load_ep(pf.ep, L, Wimg, ob, lane >> 4);
    }
}

// the k tables of the layers with a kernel > 1x1 (filled once per launch)
__device__ void rn_fill_ktabs(const RPlan& R, float* lds, int NG, int Wb, int P) {
    if (R.n_ktab == 0) return;                      // (walking the layer list costs a scalar load per layer)
    for (int i = 0; i < R.n; ++i) {
        const RLayer& L = R.L[i];
        if (L.kk == 1 || L.otab) continue;
        int* tab = reinterpret_cast<int*>(lds) + L.ktab;
        for (int k = threadIdx.x; k < L.K; k += blockDim.x) {
            const int c = k / L.kk, r = k - c * L.kk, j = r / L.kw, ii = r - j * L.kw;
            const int dx = (L.kw - 1 - ii) - L.pw, dy = (L.kh - 1 - j) - L.ph;
            const int off = c * P * NG + (dx + Wb * dy) * NG;
            tab[k] = off * 256 | ((dx + 8) << 4) | (dy + 8);
        }
    }
}

// A net: its layers one by one, a workgroup barrier after each.
// NARROW: also the 1- / 2-column-block units (the learner chain's narrow
// tiles); the wide-tile kernels keep the 3-block units only
// PF: the next layer's plan entry, first A chunk and epilogue parameters are
// loaded before each layer barrier (kernels with the register room: 512
// threads).  Layers [i0, i1) (i1 < 0: to the end).
template <bool NARROW = false, bool PF = false, int NBWMAX = 3, bool PIPE = false, bool NOKK = false,
          bool RAWTANH = false>
__device__ __forceinline__ void rn_run(const RPlan& R, const float* Wimg, const float* flat, float* lds, int NG,
                                       int Wb, int P, float bn_s, unsigned long long* st = nullptr, int i0 = 0,
                                       int i1 = -1) {
    const float bn_r = 1.0f / bn_s;
    const int wv = threadIdx.x >> 6;
    if (i1 < 0) i1 = R.n;
#ifdef MZ_STAMPS
    if (st && (threadIdx.x & 63) == 0) st[wv * 64 + 63] = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (PF) {
        if (i0 >= i1) return;
        RnPf pf;
        RLayer L = rn_layer_at(R, i0);
        rn_prefetch<NARROW, NBWMAX>(L, Wimg, flat, NG, P, pf);
        for (int i = i0; i < i1; ++i) {
            RLayer Ln;
            if (i + 1 < i1) Ln = rn_layer_at(R, i + 1);
            unsigned long long* dbg = nullptr;
#ifdef MZ_STAMPS
            if (st && i - i0 < 31) dbg = st + 1024 + 8 * (i - i0);
#endif
            rn_layer<NARROW, true, NBWMAX, PIPE, NOKK, RAWTANH>(L, Wimg, flat, lds, NG, Wb, P, bn_s, bn_r, &pf, dbg);
            if (i + 1 < i1) rn_prefetch<NARROW, NBWMAX>(Ln, Wimg, flat, NG, P, pf);
#ifdef MZ_STAMPS
            if (st && (threadIdx.x & 63) == 0 && i - i0 < 31) st[wv * 64 + 2 * (i - i0)] = __builtin_amdgcn_s_memtime();
#endif
            __syncthreads();
#ifdef MZ_STAMPS
            if (st && (threadIdx.x & 63) == 0 && i - i0 < 31) st[wv * 64 + 2 * (i - i0) + 1] = __builtin_amdgcn_s_memtime();
#endif
            L = Ln;
        }
    } else {
        for (int i = i0; i < i1; ++i) {
            unsigned long long* dbg = nullptr;
#ifdef MZ_STAMPS   // wave 0's first unit: [start, operands, chunks, epilogue] at st + 768 + 8·layer
            if (st && i - i0 < 32) dbg = st + 768 + 8 * (i - i0);
#endif
            rn_layer<NARROW, false, NBWMAX, false, NOKK, RAWTANH>(rn_layer_at(R, i), Wimg, flat, lds, NG, Wb, P, bn_s, bn_r,
                                                         nullptr, dbg);
#ifdef MZ_STAMPS
            if (st && (threadIdx.x & 63) == 0 && i - i0 < 31) st[wv * 64 + 2 * (i - i0)] = __builtin_amdgcn_s_memtime();
#endif
            __syncthreads();
#ifdef MZ_STAMPS
            if (st && (threadIdx.x & 63) == 0 && i - i0 < 31) st[wv * 64 + 2 * (i - i0) + 1] = __builtin_amdgcn_s_memtime();
#endif
        }
    }
    (void)wv;
}

// Thread layout of the staging loops: game g = tid mod NG (NG a power of
// two), features f0, f0 + fs, ... — per-game addresses are computed once and
// the unrolled loop keeps several loads in flight.
struct RnLane {
    int g, f0, fs;
};
__device__ __forceinline__ RnLane rn_lane(int NG) {
    const int lg = __ffs(NG) - 1;
    return RnLane{(int)threadIdx.x & (NG - 1), (int)threadIdx.x >> lg, (int)blockDim.x >> lg};
}
// LDS tile dst[f][NG] <- val(f) for f < n
template <class Fn>
__device__ __forceinline__ void rn_stage(float* dst, int NG, int n, const RnLane& t, Fn val) {
#pragma unroll 6
    for (int f = t.f0; f < n; f += t.fs) dst[f * NG + t.g] = val(f);
}
// put(f, src[f][g]) for f < n
template <class Fn>
__device__ __forceinline__ void rn_unstage(const float* src, int NG, int n, const RnLane& t, Fn put) {
#pragma unroll 6
    for (int f = t.f0; f < n; f += t.fs) put(f, src[f * NG + t.g]);
}
// The same for a buffer that conv layers read (feature f = p + P·c is row c,
// column p·NG + g), plain or k-blocked (mz_resnet_params.h)
__device__ __forceinline__ int rn_conv_idx(int kb, int f, int g, int NG, int P) {
    if (!kb) return f * NG + g;
    const int c = f / P, p = f - c * P;
    return rn_kb_off(c, p * NG + g, P * NG);
}
template <class Fn>
__device__ __forceinline__ void rn_stage_l(float* dst, int kb, int NG, int P, int n, const RnLane& t, Fn val) {
    if (!kb) { rn_stage(dst, NG, n, t, val); return; }
#pragma unroll 4
    for (int f = t.f0; f < n; f += t.fs) dst[rn_conv_idx(1, f, t.g, NG, P)] = val(f);
}
template <class Fn>
__device__ __forceinline__ void rn_unstage_l(const float* src, int kb, int NG, int P, int n, const RnLane& t, Fn put) {
    if (!kb) { rn_unstage(src, NG, n, t, put); return; }
#pragma unroll 4
    for (int f = t.f0; f < n; f += t.fs) put(f, src[rn_conv_idx(1, f, t.g, NG, P)]);
}

// LDS tile [f][g] (plain or k-blocked) <- row_g[f] · 2^ex(g) for f < H (H % 4 == 0,
// rows 16-byte aligned; row_g = nullptr: zeros): lane l reads the 16-byte piece
// l / NG of row l mod NG (a wave instruction: 64 bytes of each of 16 rows, where
// rn_stage's layout reads 4 bytes of each), four pieces in flight per thread;
// the LDS writes of consecutive lanes stay on consecutive games' banks
template <class ExpFn, class RowFn>
__device__ __forceinline__ void rn_stage_rows(float* dst, int kb, int NG, int P, int H, ExpFn ex, RowFn row) {
    const int H4 = H >> 2, n4 = NG * H4, nt = blockDim.x, lg = __ffs(NG) - 1;   // NG a power of two
    for (int i0 = threadIdx.x; i0 < n4; i0 += 4 * nt) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            v[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (i < n4) {
                const int g = i & (NG - 1);
                const float* r = row(g);
                if (r) v[u] = reinterpret_cast<const float4*>(r)[i >> lg];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            if (i < n4) {
                const int g = i & (NG - 1), f = (i >> lg) * 4, e = ex(g);   // x·2^e: exact
                dst[rn_conv_idx(kb, f, g, NG, P)] = ldexpf(v[u].x, e);
                dst[rn_conv_idx(kb, f + 1, g, NG, P)] = ldexpf(v[u].y, e);
                dst[rn_conv_idx(kb, f + 2, g, NG, P)] = ldexpf(v[u].z, e);
                dst[rn_conv_idx(kb, f + 3, g, NG, P)] = ldexpf(v[u].w, e);
            }
        }
    }
}

// The reverse of rn_stage_rows: row_g[f..f+3] <- LDS tile [f][g] (plain or
// k-blocked) for f < H (H % 4 == 0), each lane gathering the 16-byte piece
// l / NG of game l mod NG (conflict-free LDS reads: consecutive lanes,
// consecutive games) and handing it to put(g, piece, float4): one wave
// instruction stores 64 contiguous bytes of each of 16 rows instead of 4
// bytes (rn_unstage_l), four pieces in flight per thread
template <class PutFn>
__device__ __forceinline__ void rn_unstage_rows(const float* src, int kb, int NG, int P, int H, int t0, int G,
                                                PutFn put) {
    const int H4 = H >> 2, n4 = NG * H4, nt = blockDim.x, lg = __ffs(NG) - 1;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 4 * nt) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            if (i < n4) {
                const int g = i & (NG - 1), f = (i >> lg) * 4;
                v[u] = make_float4(src[rn_conv_idx(kb, f, g, NG, P)], src[rn_conv_idx(kb, f + 1, g, NG, P)],
                                   src[rn_conv_idx(kb, f + 2, g, NG, P)], src[rn_conv_idx(kb, f + 3, g, NG, P)]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            const int g = i & (NG - 1);
            if (i < n4 && t0 + g < G) put(g, i >> lg, v[u]);
        }
    }
}

// rn_stage_rows with the pieces from ld(g, piece) (a float4; games t0 + g >=
// G stage zeros)
template <class LdFn>
__device__ __forceinline__ void rn_stage_rows_ld(float* dst, int kb, int NG, int P, int H, int t0, int G, LdFn ld) {
    const int H4 = H >> 2, n4 = NG * H4, nt = blockDim.x, lg = __ffs(NG) - 1;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 4 * nt) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            const int g = i & (NG - 1);
            v[u] = i < n4 && t0 + g < G ? ld(g, i >> lg) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * nt;
            if (i < n4) {
                const int g = i & (NG - 1), f = (i >> lg) * 4;
                dst[rn_conv_idx(kb, f, g, NG, P)] = v[u].x;
                dst[rn_conv_idx(kb, f + 1, g, NG, P)] = v[u].y;
                dst[rn_conv_idx(kb, f + 2, g, NG, P)] = v[u].z;
                dst[rn_conv_idx(kb, f + 3, g, NG, P)] = v[u].w;
            }
        }
    }
}

// 16-byte write-through (sc1) store / load of a float4 at byte offset `off`
// of buffer `rs`: the payload of a cross-workgroup hand-off (mz_poll_ge's R1
// protocol) in whole 16-byte pieces, 64 contiguous bytes per row per wave
// instruction (one 4-byte agent-scope store per element wrote each element's
// line through separately: 25 MB of writes per configs[2] launch)
typedef unsigned rn_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void rn_st_sc1(__amdgpu_buffer_rsrc_t rs, int off, float4 v) {
    const rn_v4u u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);
}
__device__ __forceinline__ float4 rn_ld_sc1(__amdgpu_buffer_rsrc_t rs, int off) {
    const rn_v4u u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}

// Batched forward of one net (mz_net_forward): x (in_feat, n) -> out0, out1.
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_rnet_forward_kernel(RNetParams Q) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& R = *Q.plan;
    const int NG = Q.ng, t0 = blockIdx.x * NG;
    rn_fill_ktabs(R, lds, NG, Q.W, Q.P);
    const RnLane t = rn_lane(NG);
    const bool ok = t0 + t.g < Q.n_items;
    {
        const float* x = Q.x + (size_t)(ok ? t0 + t.g : 0) * R.in_feat;
        rn_stage_l(lds + R.in_off, R.in_kb, NG, Q.P, R.in_feat, t, [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run(R, Q.Wimg, Q.flat, lds, NG, Q.W, Q.P, Q.bn_s);
    if (ok) {
        float* o = Q.out0 + (size_t)(t0 + t.g) * R.out0_n;
        rn_unstage_l(lds + R.out0_off, R.out0_kb, NG, Q.P, R.out0_n, t, [&](int f, float v) { o[f] = v; });
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
// exploration noise, per-game state.  GW lanes per game (A <= GW).
template <int GW>
__device__ __forceinline__ void rsearch_root_body(const RSearchParams& P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = P.plans[MZ_NET_REPR];
    const RPlan& Rp = P.plans[MZ_NET_PRED];
    const int NG = P.ng, t0 = blockIdx.x * NG, H = P.H, A = P.A;
    const int nplan = Rr.lds_floats > Rp.lds_floats ? Rr.lds_floats : Rp.lds_floats;
    float* stg = lds + nplan;                       // [16][GW] softmax / noise staging
    float* noise = stg + 16 * GW;                   // [16][GW]
    rn_fill_ktabs(Rr, lds, NG, P.W, P.P);
    const RnLane t = rn_lane(NG);
    const bool ok = t0 + t.g < P.G;
    {
        const float* x = P.obs + (size_t)(ok ? t0 + t.g : 0) * P.obs_feat;
        rn_stage_l(lds + Rr.in_off, Rr.in_kb, NG, P.P, Rr.in_feat, t, [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run(Rr, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s);                    // :234
    float* h0 = P.hid + (size_t)(ok ? t0 + t.g : 0) * (P.S + 1) * H;
    if (ok) rn_unstage_l(lds + Rr.out0_off, Rr.out0_kb, NG, P.P, H, t, [&](int f, float v) { h0[f] = v; });
    __syncthreads();
    rn_stage_l(lds + Rp.in_off, Rp.in_kb, NG, P.P, H, t, [&](int f) { return ok ? h0[f] : 0.0f; });   // prediction input = h0
    __syncthreads();
    rn_run(Rp, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s);                    // :239
    const int gl = threadIdx.x / GW, a = threadIdx.x % GW, gg = t0 + gl;
    const bool active = gl < NG && gg < P.G;
    if (active) {
        uint32_t legal = 0;
        for (int b = 0; b < A; ++b) if (P.legal[(size_t)gg * A + b]) legal |= 1u << b;
        const uint32_t gid = P.game_offset + (uint32_t)gg;
        TreeView tree = rs_tree(P, gg);
        const float prior = double_softmax_prior<GW>(a < A ? lds[Rp.out1_off + a * NG + gl] : 0.0f, a, A, legal,
                                                     stg + GW * gl);
        init_edges(tree, 0, a, A, prior);                                       // :245
        if (P.exploration) {                                                    // :247-249
            const float nz = root_noise_lane<GW>(legal, a, A, P.seed, gid, P.rng_step, P.dirichlet_alpha,
                                                 noise + GW * gl);
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
            P.hk[(size_t)gg * (P.S + 1)] = 0;                                   // h0 not used yet
        }
    }
}
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_rsearch_root(RSearchParams P) { rsearch_root_body<16>(P); }
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_rsearch_root32(RSearchParams P) { rsearch_root_body<32>(P); }

// Tree step s: expand + backup of simulation s-1 (s > 0), then select +
// gather for simulation s (s < S), or the search statistics and the action
// (s == S).  GW lanes per game, 256 / GW games per workgroup.
template <int GW>
__device__ __forceinline__ void rsearch_tree_body(const RSearchParams& P) {
    __shared__ float stg[256];
    const int gl = threadIdx.x / GW, a = threadIdx.x % GW, lane = threadIdx.x & 63;
    const int gg = blockIdx.x * (256 / GW) + gl;
    if (gg >= P.G) return;                          // whole GW-lane groups leave together
    const int A = P.A, H = P.H, S = P.S, PS = 2 * (S + 2);
    int* st = P.gst + (size_t)gg * RG_INTS;
    int* path = P.path + (size_t)gg * PS;
    TreeView tree = rs_tree(P, gg);
    const uint32_t legal = (uint32_t)st[RG_LEGAL];
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    if (P.s > 0) {
        const int e_new = P.s;                      // the node simulation s-1 expanded (:280)
        const float prior = double_softmax_prior<GW>(a < A ? P.o_logit[(size_t)gg * A + a] : 0.0f, a, A, legal,
                                                     stg + GW * gl);
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
        backup_path<GW>(tree, path, depth, P.o_v[gg], tl, A, P.players, P.discount, rN, rW, st[RG_ROOT_TP], mmin,
                        mmax, a);                                               // :281
        __builtin_amdgcn_wave_barrier();
        if (a == 0) {
            st[RG_ROOTN] = rN; st[RG_ROOTW] = __float_as_int(rW);
            st[RG_MMIN] = __float_as_int(mmin); st[RG_MMAX] = __float_as_int(mmax);
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
    }
    if (P.s < S) {
        const SelectOut so = select_path<false, GW>(tree, path, st[RG_ROOTN], st[RG_ROOT_TP], legal,
                                                __int_as_float(st[RG_MMIN]), __int_as_float(st[RG_MMAX]), a, lane,
                                                A, P.players, P.discount, nullptr, P.pbc_tab, P.sqrt_tab, P.seed,
                                                gid, P.rng_step, P.s);                    // :256-268
        if (a == 0) {
            st[RG_LEAF_E] = so.leaf_e; st[RG_LEAF_A] = so.leaf_a; st[RG_VTP] = so.vtp; st[RG_DEPTH] = so.depth;
            int* hk = P.hk + (size_t)gg * (S + 1) + so.leaf_e;   // the parent's h *= 2 in place (Q1): counted
            const int k = *hk;
            st[RG_XK] = k;
            *hk = k + 1;
        }
    } else {                                        // store_search_stats! (:115-122) + select_action (:293-306)
        const bool lg = a < A && ((legal >> a) & 1u);
        const int Nc = lg ? (int)(tree.nc(a) & 0xffffu) : 0;
        const int sum = gisum<GW>(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
        const int act = select_action_dev<GW>(Nc, legal, A, P.temp_g ? P.temp_g[gg] : P.temperature, r);
        if (a == 0) {
            const int rN = st[RG_ROOTN];
            P.root_value[gg] = rN == 0 ? 0.0f : __int_as_float(st[RG_ROOTW]) / (float)rN;
            P.action_out[gg] = act + 1;
        }
    }
}
extern "C" __global__ __launch_bounds__(256) void mz_rsearch_tree(RSearchParams P) { rsearch_tree_body<16>(P); }
extern "C" __global__ __launch_bounds__(256) void mz_rsearch_tree32(RSearchParams P) { rsearch_tree_body<32>(P); }

// Copy n units of `size` bytes (4 or 16) from global `src` to LDS `dst` with
// LDS-DMA (global_load_lds): per instruction the wave moves 64 units to the
// wave-uniform base dst + 64·c, lane l's unit landing at base + l·size.
// Issue only; the caller waits (vmcnt) before reading.
template <int SZ>
__device__ __forceinline__ void glds_copy(const void* src, void* dst, int n, int lane) {
    const char* s = reinterpret_cast<const char*>(src);
    char* d = reinterpret_cast<char*>(dst);
    for (int c = 0; c < n; c += 64)
        if (c + lane < n) {
            auto* g = (__attribute__((address_space(1))) void*)(s + (size_t)(c + lane) * SZ);
            auto* l = (__attribute__((address_space(3))) void*)(d + (size_t)c * SZ);
            if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
            else __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
        }
}

// The tree step of rsearch_tree_body with each game's tree cached in LDS for
// the launch.  A launch walks up to depth levels of select and of backup, one
// dependent access each; on the HBM tree every one of them is a cache miss
// (the previous launch wrote the records), so a deep 1-player search (BASELINE
// configs[4]: mean depth 49) spent ~2 µs per level.  Here one wave (64/GW
// games) first copies, by LDS-DMA, each game's existing nodes (edge records,
// rewards, to_play), its path and the pUCT tables into LDS, all in flight at
// once; expand, backup, select and the search statistics then run on LDS
// exactly as in rsearch_tree_body.  HBM stays the tree's home between
// launches: the records this step changed — the new node's A edges, the path
// edges backup updated, the new node's reward and to_play — are written back.
#ifdef MZ_STAMPS   // diagnostic build only: phase ticks of workgroup 0 at every 4th simulation
#define RT_STAMP(k)                                                                                   \
    do {                                                                                              \
        if (blockIdx.x == 0 && threadIdx.x == 0 && (P.s & 3) == 0)                                    \
            P.stamps[1024 + (P.s >> 2) * 16 + (k)] = __builtin_amdgcn_s_memtime();                    \
    } while (0)
#else
#define RT_STAMP(k) do {} while (0)
#endif
// RT_WAVES (mz_resnet_params.h) waves per workgroup: wave 0 walks the trees
// (expand, backup, select, the search statistics); every wave shares the
// copies in, the cached select's recompute rows and the hidden-state gather.
// The LDS trees already hold a CU alone, so the other waves cost no occupancy.
#ifndef RT_RECOMP_U
#define RT_RECOMP_U 4                               // recompute rows per group and pass
#endif
template <int GW>
__device__ __forceinline__ void rsearch_tree_lds_body(const RSearchParams& P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // per game of the workgroup: rows to recompute, moved, depth, the select's
    // start level (atomicMin over the rows), the tag, the selected leaf's parent
    __shared__ int sh_rows[4], sh_moved[4], sh_depth[4], sh_skip[4];
    __shared__ uint32_t sh_ver[4];
    __shared__ float sh_mm[4][2];                   // min / max after the backup
    RT_STAMP(0);
    constexpr int NGW = 64 / GW;
    const int tid = threadIdx.x, wave = tid >> 6, nwv = blockDim.x >> 6;
    const int lane = tid & 63, gl = lane / GW, a = lane % GW;
    const int gg = blockIdx.x * NGW + gl;
    const int A = P.A, H = P.H, S = P.S, PS = 2 * (S + 2), s = P.s;
    const int E = (S + 1) * A, NN = S + 1;
    const RsTreeLds L = rs_tree_lds(S, P.tree_game_bytes, GW);
    char* lb = reinterpret_cast<char*>(lds);
    double* pbc = reinterpret_cast<double*>(lb);
    double* sqt = pbc + (S + 2);
    // per-game state and network outputs: plain loads, issued before the copies
    const bool live = gg < P.G;
    const int gc = live ? gg : P.G - 1;
    int* st = P.gst + (size_t)gc * RG_INTS;
    const int4 st0 = reinterpret_cast<const int4*>(st)[0], st1 = reinterpret_cast<const int4*>(st)[1];
    const int4 st2 = reinterpret_cast<const int4*>(st)[2];
    const float logit = wave == 0 && s > 0 && a < A ? P.o_logit[(size_t)gc * A + a] : 0.0f;
    const float o_r = wave == 0 && s > 0 ? P.o_r[gc] : 0.0f, o_v = wave == 0 && s > 0 ? P.o_v[gc] : 0.0f;
    // LDS-DMA, the arrays dealt round the waves: tables, then per game the
    // existing nodes 0..n_old-1, the path, the cache entries and N per node
    const int n_old = s > 0 ? s : 1;
    {
        // the copies go to waves 1.. (wave 0 issues none, so its own loads above
        // complete on their own and it forms the expansion's prior under the copies)
        const int nq = nwv > 1 ? nwv - 1 : 1, wq = nwv > 1 ? wave - 1 : wave;
        int k = 0;
        auto job = [&](auto fn) { if (k++ % nq == wq) fn(); };
        job([&] { glds_copy<4>(P.pbc_tab, pbc, 2 * (S + 2), lane); });
        job([&] { glds_copy<4>(P.sqrt_tab, sqt, 2 * (S + 2), lane); });
        for (int g = 0; g < NGW; ++g) {
            const int gq = blockIdx.x * NGW + g;
            if (gq >= P.G) break;
            const char* src = P.tree + (size_t)gq * P.tree_game_bytes;
            char* dst = lb + L.tables + g * L.game;
            // the edge records in up to nwv pieces of whole 64-record instructions
            const int ne = n_old * A, per = ((ne + nq * 64 - 1) / (nq * 64)) * 64;
            for (int c0 = 0; c0 < ne; c0 += per)
                job([&] { glds_copy<16>(src + 16 * (size_t)c0, dst + 16 * (size_t)c0, ne - c0 < per ? ne - c0 : per, lane); });
            job([&] { glds_copy<4>(src + 16 * (size_t)E, dst + 16 * (size_t)E, n_old, lane); });          // nr
            job([&] { glds_copy<4>(src + 16 * (size_t)E + 4 * (size_t)NN, dst + 16 * (size_t)E + 4 * (size_t)NN,
                                   (n_old + 3) / 4, lane); });                                        // ntp (as dwords)
            job([&] { glds_copy<4>(P.path + (size_t)gq * PS, dst + L.path, PS, lane); });
            if (s > 0) {
                job([&] { glds_copy<4>(P.cache + (size_t)gq * NN, dst + L.cache, 2 * n_old, lane); });
                job([&] { glds_copy<4>(P.nN + (size_t)gq * NN, dst + L.nn, n_old, lane); });
            }
        }
    }
    char* gb = lb + L.tables + gl * L.game;
    // wave 0: double softmax of the leaf's logits (expand_node!, :88-96) for
    // simulation s-1's node, while the other waves' copies land
    float prior = 0.0f;
    if (wave == 0 && live && s > 0)
        prior = double_softmax_prior<GW>(logit, a, A, (uint32_t)st0.x, reinterpret_cast<float*>(gb + L.stg));
    RT_STAMP(1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    RT_STAMP(2);
    TreeView tree = tree_view(gb, E, NN);
    int* path = reinterpret_cast<int*>(gb + L.path);
    uint2* cache = reinterpret_cast<uint2*>(gb + L.cache);
    uint2* lvl = reinterpret_cast<uint2*>(gb + L.lvl);
    int* nn = reinterpret_cast<int*>(gb + L.nn);
    uint2* cache_g = P.cache + (size_t)gc * NN;
    const uint32_t legal = (uint32_t)st0.x;
    const int root_tp = st0.y;
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    int rN = st0.z;
    float rW = __int_as_float(st0.w), mmin = __int_as_float(st1.x), mmax = __int_as_float(st1.y);
    // ---- wave 0: expand + backup of simulation s-1 (:280-281)
    if (wave == 0 && live) {
        TreeView gt = rs_tree(P, gg);
        float* stg = reinterpret_cast<float*>(gb + L.stg);
        uint32_t ver = s > 0 ? (uint32_t)st2.z : 1u;    // the cached select's tag (RG_VER)
        int rows = 0, moved = 0, depth = 0;
        if (s == 0) {                                   // a new search: no entry is current
            if (a == 0) { cache[0] = make_uint2(0u, 0u); st[RG_VER] = 1; }
        } else {
            const int e_new = s;                        // the node simulation s-1 expanded (:280)
            init_edges(tree, e_new, a, A, prior);
            const int tl = st2.x;
            depth = st2.y;
            if (a == 0) {
                const int li = st1.z * A + st1.w;
                tree.nc(li) = (tree.nc(li) & 0xffffu) | ((uint32_t)(e_new + 1) << 16);
                tree.nr[e_new] = o_r;
                tree.ntp[e_new] = (int8_t)tl;
                path[2 * depth + 1] = e_new;
                P.path[(size_t)gg * PS + 2 * depth + 1] = e_new;   // (a skip-ahead may keep this level)
                gt.nr[e_new] = o_r;
                gt.ntp[e_new] = (int8_t)tl;
            }
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            RT_STAMP(3);
            const uint32_t omin = __float_as_uint(mmin), omax = __float_as_uint(mmax);
            if (P.players == 1)
                backup_path_1p<GW>(tree, path, depth, o_v, P.discount, rN, rW, mmin, mmax, a,
                                   reinterpret_cast<float*>(gb + L.rr), reinterpret_cast<float*>(gb + L.vin), lvl, nn);
            else
                backup_path<GW>(tree, path, depth, o_v, tl, A, P.players, P.discount, rN, rW, root_tp, mmin, mmax,
                                a, lvl, nn);                                    // :281
            // the min / max moved: every entry is stale (the tag is bumped) and
            // every expanded node is recomputed; else the path's nodes
            moved = __float_as_uint(mmin) != omin || __float_as_uint(mmax) != omax;
            ver += moved ? 1u : 0u;
            rows = s < S ? (moved ? e_new + 1 : depth + 1) : 0;
            // write-back: the new node's edges, the path edges, N per path node
            if (a < A) gt.e[e_new * A + a] = tree.e[e_new * A + a];
            for (int d = 1 + a; d <= depth; d += GW) {
                const int i = path[2 * d];
                gt.e[i] = tree.e[i];
            }
            for (int d = a; d <= depth; d += GW) {
                const uint2 l = lvl[d];
                P.nN[(size_t)gg * NN + l.x] = (int)l.y;
            }
            if (a == 0) {
                st[RG_ROOTN] = rN; st[RG_ROOTW] = __float_as_int(rW);
                st[RG_MMIN] = __float_as_int(mmin); st[RG_MMAX] = __float_as_int(mmax);
                st[RG_VER] = (int)ver;
            }
            RT_STAMP(4);
        }
        if (a == 0) {
            sh_rows[gl] = rows; sh_moved[gl] = moved; sh_depth[gl] = depth; sh_ver[gl] = ver;
            sh_mm[gl][0] = mmin; sh_mm[gl][1] = mmax;
            sh_skip[gl] = moved ? 0 : depth;            // the leaf's level always counts
        }
    }
    __syncthreads();
    // ---- every wave: the cached select's entries (mz_tree_device.h
    // select_path_cached) of the nodes whose argmax this backup can have
    // changed — the path's, or every expanded node's when min / max moved —
    // U rows per group and pass, rows dealt round the waves; the entries go to
    // LDS and to their HBM home.  A path row whose choice leaves the last path
    // (or ties) bounds the next walk's start: the levels above it are retraced.
    const int rows = live ? sh_rows[gl] : 0;
    if (rows > 0) {
        const bool moved = sh_moved[gl] != 0;
        const int depth = sh_depth[gl];
        const uint32_t ver = sh_ver[gl];
        const float mn = sh_mm[gl][0], mx = sh_mm[gl][1];
        const bool lg = a < A && ((legal >> a) & 1u);
        constexpr int U = RT_RECOMP_U;
        int Dl = depth;
        for (int j0 = wave * U; j0 < rows; j0 += nwv * U) {
            int slot[U], Np[U], ch[U];
            bool act[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = j0 + u;
                act[u] = j < rows;
                const int jc = act[u] ? j : 0;
                if (moved) { slot[u] = jc; Np[u] = nn[jc]; }
                else { const uint2 l = lvl[jc]; slot[u] = (int)l.x; Np[u] = (int)l.y; }
            }
            // the pUCT prior factor from the pb_term triangle in global memory
            // (L2-resident; its loads overlap across the rows) instead of an f64
            // division per child
            cache_rows<GW, true, U>(tree, cache, ver, slot, Np, act, lg, a, A, mn, mx, P.pbterm, lane, nullptr,
                                    nullptr, cache_g, ch);
            if (!moved) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = j0 + u;
                    if (j < depth && ch[u] != path[2 * (j + 1)] - slot[u] * A) Dl = Dl < j ? Dl : j;
                }
            }
        }
        if (!moved && a == 0 && Dl < depth) atomicMin(sh_skip + gl, Dl);
    }
    __syncthreads();
    RT_STAMP(5);
#ifdef MZ_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0 && (P.s & 3) == 0) {
        P.stamps[1024 + (P.s >> 2) * 16 + 10] = sh_moved[0];
        P.stamps[1024 + (P.s >> 2) * 16 + 11] = (unsigned long long)sh_depth[0];
        P.stamps[1024 + (P.s >> 2) * 16 + 12] = (unsigned long long)sh_skip[0];
    }
#endif
    RT_STAMP(6);
    if (s < S) {
        // ---- wave 0: select (:256-268), the walk from level D: its node and
        // the nc word of the edge into it from this game's path (levels 0..D of
        // the HBM path stay as they are)
        if (wave == 0 && live) {
            int D = sh_skip[gl];
            if (sh_moved[gl] != 0 && !P.no_moved_skip) {
                // min / max moved: every expanded node's entry was just recomputed
                // (current tag), so the walk from the root retraces the last path
                // down to the first level whose new entry leaves it (or ties)
                const int depth = sh_depth[gl];
                const uint32_t ver = sh_ver[gl];
                int Dl = depth;
                for (int j = a; j < depth; j += GW) {
                    const int node = (int)lvl[j].x;
                    const uint2 ce = cache[node];
                    const bool on = (ce.x >> 5) == ver && (int)(ce.x & 31u) == path[2 * (j + 1)] - node * A;
                    if (!on && j < Dl) Dl = j;
                }
#pragma unroll
                for (int o = GW / 2; o > 0; o >>= 1) { const int t = __shfl_xor(Dl, o); Dl = t < Dl ? t : Dl; }
                D = Dl;
            }
            const int e0 = D > 0 ? path[2 * D + 1] : 0;
            const uint32_t npc0 = D > 0 ? tree.nc(path[2 * D]) : 0u;
            const SelectOut so = select_path_cached<GW, false>(tree, cache, sh_ver[gl], P.path + (size_t)gg * PS, rN,
                                                               root_tp, legal, mmin, mmax, a, lane, A, P.players,
                                                               nullptr, P.seed, gid, P.rng_step, s, pbc, sqt, D, e0,
                                                               npc0);
            if (a == 0) {
                st[RG_LEAF_E] = so.leaf_e; st[RG_LEAF_A] = so.leaf_a; st[RG_VTP] = so.vtp; st[RG_DEPTH] = so.depth;
                int* hk = P.hk + (size_t)gg * (S + 1) + so.leaf_e;   // the parent's h *= 2 in place (Q1): counted
                const int k = *hk;
                st[RG_XK] = k;
                *hk = k + 1;
            }
        }
        RT_STAMP(7);
        RT_STAMP(8);
    } else if (wave == 0 && live) {                 // store_search_stats! (:115-122) + select_action (:293-306)
        const bool lg = a < A && ((legal >> a) & 1u);
        const int Nc = lg ? (int)(tree.nc(a) & 0xffffu) : 0;
        const int sum = gisum<GW>(Nc);
        if (a < A) P.child_visits[(size_t)gg * A + a] = lg ? (float)((double)Nc / (double)sum) : 0.0f;
        const uint32_t r = mz_rng_u32(P.seed, MZ_RNG_ACTION, gid, P.rng_step, 0);
        const int act = select_action_dev<GW>(Nc, legal, A, P.temp_g ? P.temp_g[gg] : P.temperature, r);
        if (a == 0) {
            P.root_value[gg] = rN == 0 ? 0.0f : rW / (float)rN;
            P.action_out[gg] = act + 1;
        }
    }
}
extern "C" __global__ __launch_bounds__(64 * RT_WAVES) void mz_rsearch_tree_lds(RSearchParams P) {
    rsearch_tree_lds_body<16>(P);
}
extern "C" __global__ __launch_bounds__(64 * RT_WAVES) void mz_rsearch_tree_lds32(RSearchParams P) {
    rsearch_tree_lds_body<32>(P);
}

// Networks of simulation s: blockIdx.y = 0 prediction(parent h), 1 dynamics
// (2h ⊕ a/|A|, Q1) writing h' into hidden slot s+1.  With P.rew_split the
// dynamics is y = 0 (the producer, dispatched first: no consumer can occupy
// the CU its producer needs) and the prediction workgroup of the tile runs the
// dynamics reward head after its own heads, on the published trunk output.
extern "C" __global__ __launch_bounds__(RN_THREADS_NETS) void mz_rsearch_nets(RSearchParams P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const bool split = P.rew_split != 0;
    const int net = (blockIdx.y == 0) != split ? MZ_NET_PRED : MZ_NET_DYN;
#ifdef RN_DIAG_ONLY          // diagnostic builds (wrong results): time one net alone
    if ((int)blockIdx.y != RN_DIAG_ONLY) return;
#endif
    const RPlan& R = P.plans[net];
    const int NG = P.ng, t0 = blockIdx.x * NG, H = P.H, S = P.S;
    unsigned long long* st = nullptr;
#ifdef MZ_STAMPS
    if (P.stamps && blockIdx.x == 0 && P.s == 0) st = P.stamps + blockIdx.y * 1024;   // 12 waves x 64
    if (st && (threadIdx.x & 63) == 0) st[(threadIdx.x >> 6) * 64 + 60] = __builtin_amdgcn_s_memtime();
#endif
    rn_fill_ktabs(R, lds, NG, P.W, P.P);
    const RnLane t = rn_lane(NG);
    const int gg = t0 + t.g;
    const bool ok = gg < P.G;
    // prediction(parent h) and dynamics(2h ⊕ a/|A|) read the parent's stored h'
    // (hid[leaf_e]) times 2^hk and 2^(hk+1): the value make_state_action (Q1)
    // leaves in place after the node's hk earlier uses, and the doubled value of
    // this use, bit for bit (powers of two are exact; RSearchParams::hk).  The
    // dynamics' a/|A| plane (features H .. in_feat - 1): the leaf actions are
    // loaded first, so their latency overlaps the row loads; a/|A| as the host's
    // table, (float)((a + 1) / |A|) in f64
    const int np = R.in_feat - H, npl = net == MZ_NET_DYN ? NG * np : 0;
    int la = 0;
    if ((int)threadIdx.x < npl) {
        const int gq = t0 + (int)threadIdx.x / np;
        if (gq < P.G) la = P.gst[(size_t)gq * RG_INTS + RG_LEAF_A];
    }
    const int e1 = net == MZ_NET_DYN ? 1 : 0;
    if ((H & 3) == 0) {
        rn_stage_rows(lds + R.in_off, R.in_kb, NG, P.P, H,
                      [&](int g) { return t0 + g < P.G ? P.gst[(size_t)(t0 + g) * RG_INTS + RG_XK] + e1 : 0; },
                      [&](int g) -> const float* {
                          if (t0 + g >= P.G) return nullptr;
                          const int sl = P.gst[(size_t)(t0 + g) * RG_INTS + RG_LEAF_E];
                          return P.hid + ((size_t)(t0 + g) * (S + 1) + sl) * H;
                      });
    } else {
        const int* q = P.gst + (size_t)(ok ? gg : 0) * RG_INTS;
        const float* x = P.hid + ((size_t)(ok ? gg : 0) * (S + 1) + q[RG_LEAF_E]) * H;
        const int e = q[RG_XK] + e1;
        rn_stage_l(lds + R.in_off, R.in_kb, NG, P.P, H, t, [&](int f) { return ok ? ldexpf(x[f], e) : 0.0f; });
    }
    for (int i = threadIdx.x; i < npl; i += blockDim.x) {
        const int g = i / np, f = H + (i - g * np);
        if (i >= (int)blockDim.x && t0 + g < P.G) la = P.gst[(size_t)(t0 + g) * RG_INTS + RG_LEAF_A];
        const float av = t0 + g < P.G ? (float)((double)(la + 1) / (double)P.A) : 0.0f;
        lds[R.in_off + rn_conv_idx(R.in_kb, f, g, NG, P.P)] = av;
    }
    __syncthreads();
    // prediction / dynamics: 1x1 convs and Dense layers only (rn_specs), so
    // the k-table path is left out of this kernel (registers: the 12-wave cap)
    // (the PF prefetch set does not fit the 12-wave register budget: 200 spilled VGPRs, and an A-only
    // prefetch into the layer's own registers measured 76 vs 70 µs)
    if (split) {
        if (net == MZ_NET_DYN) {
            rn_run<false, false, 3, false, true, true>(R, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s, st, 0, P.trunk_nl);
            const RLayer Ls = rn_layer_at(R, P.dyn_split);             // the reward head's input: the trunk output
            if ((H & 3) == 0) {                                         // 16-byte sc1 pieces (rn_st_sc1)
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(P.trunk, (short)0, P.G * H * 4, 0x00020000);
                rn_unstage_rows(lds + Ls.in_off, Ls.in_kb, NG, P.P, H, t0, P.G, [&](int g, int q, float4 v) {
                    rn_st_sc1(rs, ((t0 + g) * H + 4 * q) * 4, v);
                });
            } else if (ok) {
                rn_unstage_l(lds + Ls.in_off, Ls.in_kb, NG, P.P, H, t, [&](int f, float v) {
                    __hip_atomic_store(P.trunk + (size_t)gg * H + f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                });
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // every wave's stores performed
            __syncthreads();
            if (threadIdx.x == 0 && (int)blockIdx.x != P.dbg_skip)
                __hip_atomic_store(P.tprog + blockIdx.x, P.tepoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            rn_run<false, false, 3, false, true, true>(R, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s, nullptr, P.trunk_nl,
                                                 P.dyn_split);                        // the state head
            if ((H & 3) == 0) {
                rn_unstage_rows(lds + R.out0_off, R.out0_kb, NG, P.P, H, t0, P.G, [&](int g, int q, float4 v) {
                    reinterpret_cast<float4*>(P.hid + ((size_t)(t0 + g) * (S + 1) + P.s + 1) * H)[q] = v;
                });
            } else if (ok) {
                float* o = P.hid + ((size_t)gg * (S + 1) + P.s + 1) * H;
                rn_unstage_l(lds + R.out0_off, R.out0_kb, NG, P.P, H, t, [&](int f, float v) { o[f] = v; });
            }
            if ((int)threadIdx.x < NG && t0 + (int)threadIdx.x < P.G)     // the new node's h' not used yet
                P.hk[(size_t)(t0 + threadIdx.x) * (S + 1) + P.s + 1] = 0;
            return;
        }
        rn_run<false, false, 3, false, true, true>(R, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s, st);
        if (ok) {
            if (t.f0 == 0) P.o_v[gg] = rn_act(R.out0_act, lds[R.out0_off + t.g]);   // (RAWTANH)
            float* o = P.o_logit + (size_t)gg * P.A;
            rn_unstage(lds + R.out1_off, NG, P.A, t, [&](int f, float v) { o[f] = v; });
        }
        __syncthreads();                                              // the outputs read before the LDS is reused
        if (threadIdx.x == 0)                   // bounded: a publish that never comes is reported (P.fault)
            mz_poll_ge(P.tprog + blockIdx.x, P.tepoch, P.fault, MZ_FAULT_RS_TRUNK, P.poll_ticks);
        __syncthreads();
        const RPlan& Rd = P.plans[MZ_NET_DYN];
        const RLayer Ls = rn_layer_at(Rd, P.dyn_split);
        if ((H & 3) == 0) {                                           // 16-byte sc1 pieces (rn_ld_sc1)
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(P.trunk, (short)0, P.G * H * 4, 0x00020000);
            rn_stage_rows_ld(lds + Ls.in_off, Ls.in_kb, NG, P.P, H, t0, P.G, [&](int g, int q) {
                return rn_ld_sc1(rs, ((t0 + g) * H + 4 * q) * 4);
            });
        } else {
            rn_stage_l(lds + Ls.in_off, Ls.in_kb, NG, P.P, H, t, [&](int f) {
                return ok ? __hip_atomic_load(P.trunk + (size_t)gg * H + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : 0.0f;
            });
        }
        __syncthreads();
        rn_run<false, false, 3, false, true, true>(Rd, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s, nullptr, P.dyn_split);
        if (ok && t.f0 == 0) P.o_r[gg] = rn_act(Rd.out1_act, lds[Rd.out1_off + t.g]);
        return;
    }
    rn_run<false, false, 3, false, true, true>(R, P.Wimg, P.flat, lds, NG, P.W, P.P, P.bn_s, st);
#ifdef MZ_STAMPS
    if (st && (threadIdx.x & 63) == 0) st[(threadIdx.x >> 6) * 64 + 61] = __builtin_amdgcn_s_memtime();
#endif
    if (!ok) return;
    if (net == MZ_NET_PRED) {
        if (t.f0 == 0) P.o_v[gg] = rn_act(R.out0_act, lds[R.out0_off + t.g]);
        float* o = P.o_logit + (size_t)gg * P.A;
        rn_unstage(lds + R.out1_off, NG, P.A, t, [&](int f, float v) { o[f] = v; });
    } else {
        float* o = P.hid + ((size_t)gg * (S + 1) + P.s + 1) * H;
        rn_unstage_l(lds + R.out0_off, R.out0_kb, NG, P.P, H, t, [&](int f, float v) { o[f] = v; });
        if (t.f0 == 0) P.o_r[gg] = rn_act(R.out1_act, lds[R.out1_off + t.g]);
        if (t.f0 == 0) P.hk[(size_t)gg * (S + 1) + P.s + 1] = 0;   // the new node's h' not used yet
    }
}

// ================================================================ learner
// Forward unroll of the learner (Learning.jl:347-370): representation, then
// for i = 1..K prediction(h_{i-1}) -> step i (step 0 is the same prediction of
// h0, written once for both), dynamics(2h ⊕ a_i/|A|) -> h_i, r_i; r_0 = 0.
// The parameters of this workgroup's step in a multi-step launch (U.ms > 0,
// blockIdx.z = the step; RUnrollParams.ms), else U itself
__device__ __forceinline__ RUnrollParams rn_step(const RUnrollParams& U, int zs = -1) {
    RUnrollParams V = U;
    if (U.ms) {
        const size_t z = zs >= 0 ? (size_t)zs : blockIdx.z, B = (size_t)U.B;
        V.Wimg += z * U.ms_wimg; V.flat += z * U.ms_flat;
        V.obs += z * U.ms_obs; V.actions += z * U.ms_k1;
        V.pv += z * U.ms_k1; V.pp += z * U.ms_tp; V.pr += z * U.ms_k1;
        V.hs += z * U.ms_hs; V.ts += z * U.ms_hs; V.prog += z * B;
        V.rq.step += (uint32_t)z;
        V.rq.obs += z * U.ms_obs; V.rq.actions += z * U.ms_k1; V.rq.tv += z * U.ms_k1; V.rq.tr += z * U.ms_k1;
        V.rq.tpol += z * U.ms_tp; V.rq.gscale += z * B; V.rq.index += z * 2 * B;
    }
    return V;
}

extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_kernel(RUnrollParams U) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = U.plans[MZ_NET_REPR];
    const RPlan& Rp = U.plans[MZ_NET_PRED];
    const RPlan& Rd = U.plans[MZ_NET_DYN];
    const int NG = U.ng, t0 = blockIdx.x * NG, H = U.H, A = U.A, K1 = U.K + 1;
    const RnLane t = rn_lane(NG);
    const int b = t0 + t.g;
    const bool ok = b < U.B;
    const size_t bs = (size_t)(ok ? b : 0);
    float* hs = U.hs + bs * H;
    rn_fill_ktabs(Rr, lds, NG, U.W, U.P);
    {
        const float* x = U.obs + bs * U.obs_feat;
        rn_stage_l(lds + Rr.in_off, Rr.in_kb, NG, U.P, Rr.in_feat, t, [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run(Rr, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                     // :347
    if (ok) rn_unstage_l(lds + Rr.out0_off, Rr.out0_kb, NG, U.P, H, t, [&](int f, float v) { hs[f] = v; });
    if (ok && t.f0 == 0) U.pr[bs * K1] = 0.0f;
    const int ns = U.K > 0 ? U.K : 1;              // K = 0: the prediction of h0 alone
    for (int s = 1; s <= ns; ++s) {
        __syncthreads();
        rn_fill_ktabs(Rp, lds, NG, U.W, U.P);
        rn_stage_l(lds + Rp.in_off, Rp.in_kb, NG, U.P, H, t, [&](int f) { return ok ? hs[f] : 0.0f; });
        __syncthreads();
        rn_run(Rp, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                 // :351 / :356
        if (ok) {
            // step s (and step 0 from the same prediction of h0, Q10)
            for (int j = s == 1 ? 0 : s; j <= (s <= U.K ? s : 0); ++j) {
                if (t.f0 == 0) U.pv[bs * K1 + j] = lds[Rp.out0_off + t.g];
                float* o = U.pp + (bs * K1 + j) * A;
                rn_unstage(lds + Rp.out1_off, NG, A, t, [&](int f, float v) { o[f] = v; });
            }
        }
        if (s > U.K) break;
        __syncthreads();
        rn_fill_ktabs(Rd, lds, NG, U.W, U.P);
        {                                                                      // make_dynamics_input (:293-304)
            const float av = ok ? U.actions[bs * K1 + (s - 1)] / (float)A : 0.0f;
            rn_stage_l(lds + Rd.in_off, Rd.in_kb, NG, U.P, Rd.in_feat, t, [&](int f) { return !ok ? 0.0f : f < H ? hs[f] * 2.0f : av; });
        }
        __syncthreads();
        rn_run(Rd, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s);                 // :362
        if (ok) {
            rn_unstage_l(lds + Rd.out0_off, Rd.out0_kb, NG, U.P, H, t, [&](int f, float v) { hs[f] = v; });
            if (t.f0 == 0) U.pr[bs * K1 + s] = lds[Rd.out1_off + t.g];
        }
    }
}

// Learner unroll, split form (the same read-outs as mz_runroll_kernel, bit for
// bit: every tile column is an independent fma chain, so the tile width does
// not change a result).  The unroll's only sequential part is representation
// (:347) then the K dynamics steps' state path (:355-362: the trunk and the
// state head, h_{s-1} -> h_s); the K predictions (:351, :356) only read h_0 ..
// h_{K-1} and the K reward heads only the dynamics trunk outputs.
// mz_runroll_chain runs that path on narrow tiles of ng_l samples — B / ng_l
// workgroups instead of B / 16, a narrower MFMA column range per layer, so a
// short per-layer critical path, with each layer's plan entry and first
// operands loaded under the previous one — and stores h_s to hs[b][s] and the
// trunk output of step s to ts[b][s-1]; mz_runroll_pred then runs the B·K
// predictions (blockIdx.y = 0) and the B·K reward heads (y = 1) as one wide
// launch on tiles of ng items.
template <int NBWMAX>
__device__ __forceinline__ void runroll_chain_body(const RUnrollParams& U) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = U.plans_l[MZ_NET_REPR];
    const RPlan& Rd = U.plans_l[MZ_NET_DYN];
    const int NG = U.ng_l, t0 = blockIdx.x * NG, H = U.H, A = U.A, K = U.K, K1 = K + 1;
    const RnLane t = rn_lane(NG);
    const int b = t0 + t.g;
    const bool ok = b < U.B;
    const size_t bs = (size_t)(ok ? b : 0);
    const int KH = K > 0 ? K : 1;
    const int split = U.dyn_split;                 // first reward-head layer of the dynamics plan
    const int trunk = Rd.L[split].in_off;          // the trunk output the reward head reads
    float* hs = U.hs + bs * KH * H;                 // [K][H]: h_s, s = 0 .. K-1
    float* ts = U.ts + bs * KH * H;                 // [K][H]: trunk output of step s + 1
    unsigned long long* st_r = nullptr;
    unsigned long long* st_d = nullptr;
#ifdef MZ_STAMPS
    if (U.stamps && blockIdx.x == 0) { st_r = U.stamps; st_d = U.stamps + 512; }
#endif
    rn_fill_ktabs(Rr, lds, NG, U.W, U.P);
    if (Rr.tab_n) {                                 // the representation's offset tables (+ the zero float)
        const int4* src = reinterpret_cast<const int4*>(U.otab + Rr.tab_src);
        int4* dst = reinterpret_cast<int4*>(reinterpret_cast<int*>(lds) + Rr.tab_lds);
        for (int i = threadIdx.x; i < Rr.tab_n / 4; i += blockDim.x) dst[i] = src[i];
        if (threadIdx.x == 0) lds[Rr.zero_off] = 0.0f;
    }
    {
        const float* x = U.obs + bs * U.obs_feat;
        rn_stage_l(lds + Rr.in_off, Rr.in_kb, NG, U.P, Rr.in_feat, t, [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run<true, true, NBWMAX>(Rr, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, st_r);         // :347
    if (ok) rn_unstage_l(lds + Rr.out0_off, Rr.out0_kb, NG, U.P, H, t, [&](int f, float v) { hs[f] = v; });
    if (ok && t.f0 == 0) U.pr[bs * K1] = 0.0f;                                 // :352 zeros
    for (int s = 1; s <= K; ++s) {
        __syncthreads();
        rn_fill_ktabs(Rd, lds, NG, U.W, U.P);
        {                                                                      // make_dynamics_input (:293-304)
            const float av = ok ? U.actions[bs * K1 + (s - 1)] / (float)A : 0.0f;
            const float* hp = hs + (size_t)(s - 1) * H;
            rn_stage_l(lds + Rd.in_off, Rd.in_kb, NG, U.P, Rd.in_feat, t, [&](int f) { return !ok ? 0.0f : f < H ? hp[f] * 2.0f : av; });
        }
        __syncthreads();
        rn_run<true, true, NBWMAX>(Rd, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, s == 1 ? st_d : nullptr, 0, split);  // :362
        if (ok) {
            if (s < K) rn_unstage_l(lds + Rd.out0_off, Rd.out0_kb, NG, U.P, H, t,
                                    [&](int f, float v) { hs[(size_t)s * H + f] = v; });
            rn_unstage_l(lds + trunk, Rd.L[split].in_kb, NG, U.P, H, t, [&](int f, float v) { ts[(size_t)(s - 1) * H + f] = v; });
        }
    }
}

extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_chain(RUnrollParams U) {
    runroll_chain_body<3>(rn_step(U));
}
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_chain1(RUnrollParams U) {
    runroll_chain_body<1>(rn_step(U));
}

// ---- the chain with a register-resident dynamics path (mz_runroll_chain_r)
// The K dynamics steps run the same RD_NL trunk + state-head layers K times:
// 1x1 convs of 64 output channels (one 16-row block per wave, waves 0..3) on
// one 16-column block.  Their A fragments are loaded into registers once per
// launch (layer 0, K = nf + 1 on the plain input: two chunks; layers 1.. (K =
// 64, k-blocked input): one chunk each) and their epilogue parameters staged in
// LDS, so a layer is LDS reads, 16 MFMAs and a branch-free epilogue between two
// barriers: no plan decode through the generic layer code, no global loads.
// The arithmetic is rn_layer_t's (MODE 1 / MODE 3, NBW = 1) and
// rn_epilogue's, operation for operation.  256 threads: one wave per SIMD, so
// the resident fragments (16 floats per chunk) have the register file's room.
template <bool RES_ADD>
__device__ __forceinline__ void rd_epilogue(const RLayer& L, const mz_f32x4 (&acc)[4], const float4 (&ep)[4],
                                            const float (&res)[4], float* lds, int ob, int kl, int n, int ncols,
                                            float bn_s, float bn_r) {
    float d[4];
    bool tiny = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float t = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
        t = t + ep[r].x;
        d[r] = t;
        tiny |= !(fabsf(t) >= 0x1p-100f) || fabsf(t) == INFINITY;
    }
    float q[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float t = d[r] - 0.0f;
        const float q0 = t * bn_r;
        const float e = fmaf(-q0, bn_s, t);
        q[r] = fmaf(e, bn_r, q0);
    }
    if (__builtin_expect(__ballot(tiny) != 0, 0)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (!(fabsf(d[r]) >= 0x1p-100f) || fabsf(d[r]) == INFINITY) q[r] = (d[r] - 0.0f) / bn_s;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = ep[r].y * q[r] + ep[r].z;
    if (n < ncols) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = d[r];
            if constexpr (RES_ADD) v = v + res[r];
            lds[L.out_off + rn_out_idx(L.out_kb, ob, kl, r, n, ncols)] = mz_relu(v);
        }
    }
}

// layer I of the resident chain (wave ob < 4); a[] = this layer's chunks;
// NB column blocks of 16, one after the other (reads, 16 MFMAs, epilogue)
template <int NCH, int NB = 1>
__device__ __forceinline__ void rd_layer(const RLayer& L, const float (&a)[NCH][4][4], const float4* ep_lds,
                                         float* lds, int ncols, float bn_s, float bn_r) {
    const int lane = threadIdx.x & 63, ob = threadIdx.x >> 6, kl = lane >> 4, n = lane & 15;
    float4 ep[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ep[r] = ep_lds[ob * 16 + kl * 4 + r];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int ni = i * 16 + n;
        const int nc = ni < ncols ? ni : ncols - 1;
        float res[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            res[r] = L.res_add ? lds[L.res_off + rn_out_idx(L.res_kb, ob, kl, r, nc, ncols)] : 0.0f;
        mz_f32x4 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = mz_f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (NCH == 1) {               // MODE 3: K = 64, NQ = 4, k-blocked input
            const uint32_t b0 = (uint32_t)(L.in_off + n * 16 + 4 * (((n >> 2) & 3) ^ rn_kb_sigma(kl))) * 4u +
                                1024u * i;
            float4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                v[q] = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(lds) + b0 +
                                                        (uint32_t)(q * ncols) * 64u);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float bv = jj == 0 ? v[q].x : jj == 1 ? v[q].y : jj == 2 ? v[q].z : v[q].w;
                    acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0][q][jj], bv, acc[q], 0, 0, 0);
                }
        } else {                                // MODE 1: plain input, NQ = L.nq in (4, 4 NCH]
            const int NQ = L.nq, K = L.K;
            const int cb = L.in_off + nc;
            float b[NCH][4][4];
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int k = (q * NQ + 4 * c + jj) * 4 + kl;
                        const bool kin = k < K && 4 * c + jj < NQ;
                        const float v = lds[cb + (kin ? k : K - 1) * ncols];
                        b[c][jj][q] = kin ? v : 0.0f;
                    }
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    if (4 * c + jj >= NQ) break;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c][q][jj], b[c][jj][q], acc[q], 0, 0, 0);
                }
        }
        if (L.res_add) rd_epilogue<true>(L, acc, ep, res, lds, ob, kl, ni, ncols, bn_s, bn_r);
        else rd_epilogue<false>(L, acc, ep, res, lds, ob, kl, ni, ncols, bn_s, bn_r);
    }
}

template <int I, int NL, int NB>
__device__ __forceinline__ void rd_run(const RPlan& Rd, const float (&a0)[2][4][4], const float (&ar)[NL][4][4],
                                       const float4* ep_lds, float* lds, int ncols, float bn_s, float bn_r,
                                       unsigned long long* st, int nrun = NL) {
    if constexpr (I < NL) {
        if (I >= nrun) return;                          // (wave-uniform: the last step's trunk only)
        const RLayer L = rn_layer_at(Rd, I);
        if constexpr (I == 0) {
#ifdef MZ_STAMPS
            if (st && (threadIdx.x & 63) == 0) st[(threadIdx.x >> 6) * 64 + 63] = __builtin_amdgcn_s_memtime();
#endif
            rd_layer<2, NB>(L, a0, ep_lds, lds, ncols, bn_s, bn_r);
        } else {
            const float (&a1)[1][4][4] = *reinterpret_cast<const float (*)[1][4][4]>(&ar[I]);
            rd_layer<1, NB>(L, a1, ep_lds + I * 64, lds, ncols, bn_s, bn_r);
        }
#ifdef MZ_STAMPS
        if (st && (threadIdx.x & 63) == 0 && I < 31) st[(threadIdx.x >> 6) * 64 + 2 * I] = __builtin_amdgcn_s_memtime();
#endif
        __syncthreads();
#ifdef MZ_STAMPS
        if (st && (threadIdx.x & 63) == 0 && I < 31) st[(threadIdx.x >> 6) * 64 + 2 * I + 1] = __builtin_amdgcn_s_memtime();
#endif
        rd_run<I + 1, NL, NB>(Rd, a0, ar, ep_lds, lds, ncols, bn_s, bn_r, st, nrun);
    }
    (void)st;
}

// mz_runroll_fused_r's hand-off between workgroups, on the scoped caches of
// gfx950 without whole-L2 write-back / invalidate: the chain stores h and the
// trunk outputs as agent-scope atomics (written through to the agent's
// coherence point), every wave waits for its stores (vmcnt 0), then after the
// barrier one agent-scope store of the progress word.  An item polls the word
// with agent-scope loads (mz_poll_ge, bounded: a chain that never publishes
// sets MZ_FAULT_RD_PROGRESS, which fails the host's next synchronisation,
// instead of hanging the grid) and reads its input with agent-scope loads
// (they miss any stale L1 / L2 copy).
__device__ __forceinline__ void rd_st(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float rd_ld(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rd_publish(const RUnrollParams& U, int b, int p) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && b != U.dbg_skip)
        __hip_atomic_store(U.prog + b, U.prog_base + (unsigned long long)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef MZ_STAMPS
    if (U.stamps && threadIdx.x == 0) U.stamps[2048 + 4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}
__device__ __forceinline__ void rd_wait(const RUnrollParams& U, int b, int p) {
    if (threadIdx.x == 0) {
        mz_poll_ge(U.prog + b, U.prog_base + (unsigned long long)p, U.fault, MZ_FAULT_RD_PROGRESS, U.poll_ticks);
#ifdef MZ_STAMPS
        if (U.stamps) U.stamps[2048 + 4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    __syncthreads();
}

// NL: the dynamics chain's layers ([0, dyn_split)); NB: column blocks of the tile;
// FUSE: mz_runroll_fused_r's chain blocks (ng_l = 1: tile = sample), which
// draw their sample first when U.fuse_sample and publish their progress
template <int NL, int NB, bool FUSE = false>
__device__ __forceinline__ void runroll_chain_r_body(const RUnrollParams& U, int tile) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& Rr = U.plans_l[MZ_NET_REPR];
    const RPlan& Rd = U.plans_l[MZ_NET_DYN];
    const int NG = U.ng_l, t0 = tile * NG, H = U.H, A = U.A, K = U.K, K1 = K + 1;
    if constexpr (FUSE) {
        if (U.fuse_sample) {                                   // get_batch (ReplayBuffer.jl:188-217)
            if (threadIdx.x < 64 && t0 < U.B) rp_sample_one(U.rq, t0, threadIdx.x);
            __threadfence_block();
            __syncthreads();
        }
    }
    const RnLane t = rn_lane(NG);
    const int b = t0 + t.g;
    const bool ok = b < U.B;
    const size_t bs = (size_t)(ok ? b : 0);
    const int KH = K > 0 ? K : 1;
    const int split = U.dyn_split;
    const int trunk = Rd.L[split].in_off;
    const int ncols = U.P * NG;
    float* hs = U.hs + bs * KH * H;
    float* ts = U.ts + bs * KH * H;
    unsigned long long* st_r = nullptr;
    unsigned long long* st_d = nullptr;
#ifdef MZ_STAMPS
    if (U.stamps && tile == 0) { st_r = U.stamps; st_d = U.stamps + 512; }
#endif
    float4* ep_lds = reinterpret_cast<float4*>(lds + U.rd_ep_off);   // [NL][64] {bias, γ, β, 0}
    for (int i = threadIdx.x; i < NL * 64; i += blockDim.x) {
        const RLayer L = rn_layer_at(Rd, i >> 6);
        ep_lds[i] = reinterpret_cast<const float4*>(U.Wimg + L.ep_img)[i & 63];
    }
    rn_fill_ktabs(Rr, lds, NG, U.W, U.P);
    if (Rr.tab_n) {
        const int4* src = reinterpret_cast<const int4*>(U.otab + Rr.tab_src);
        int4* dst = reinterpret_cast<int4*>(reinterpret_cast<int*>(lds) + Rr.tab_lds);
        for (int i = threadIdx.x; i < Rr.tab_n / 4; i += blockDim.x) dst[i] = src[i];
        if (threadIdx.x == 0) lds[Rr.zero_off] = 0.0f;
    }
    {
        const float* x = U.obs + bs * U.obs_feat;
        rn_stage_l(lds + Rr.in_off, Rr.in_kb, NG, U.P, Rr.in_feat, t, [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run<true, true, NB == 1 ? 1 : 3, true>(Rr, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, st_r);   // :347
    // resident A fragments of the dynamics chain (wave w = row block w), issued
    // after the representation (live across it, they cost its code registers)
    const int lane = threadIdx.x & 63, ob = threadIdx.x >> 6;
    float a0[2][4][4], ar[NL][4][4];
    {
        const RLayer L0 = rn_layer_at(Rd, 0);
        rn_load_a(a0[0], U.Wimg, L0, ob, 0, lane);
        rn_load_a(a0[1], U.Wimg, L0, ob, 1, lane);
#pragma unroll
        for (int i = 1; i < NL; ++i) rn_load_a(ar[i], U.Wimg, rn_layer_at(Rd, i), ob, 0, lane);
    }
    if (ok) rn_unstage_l(lds + Rr.out0_off, Rr.out0_kb, NG, U.P, H, t, [&](int f, float v) {
        if constexpr (FUSE) rd_st(hs + f, v); else hs[f] = v;
    });
    if (ok && t.f0 == 0) U.pr[bs * K1] = 0.0f;                                 // :352 zeros
    if constexpr (FUSE) rd_publish(U, t0, 1);                                 // h_0
    const float bn_r = 1.0f / U.bn_s;
    for (int s = 1; s <= K; ++s) {
        __syncthreads();
        {                                                                      // make_dynamics_input (:293-304)
            const float av = ok ? U.actions[bs * K1 + (s - 1)] / (float)A : 0.0f;
            const float* hp = hs + (size_t)(s - 1) * H;
            rn_stage_l(lds + Rd.in_off, Rd.in_kb, NG, U.P, Rd.in_feat, t, [&](int f) { return !ok ? 0.0f : f < H ? hp[f] * 2.0f : av; });
        }
        __syncthreads();
        // :362, [0, split); the last step's state head is skipped: h_K is never read
        // (predictions take h_0..h_{K-1}, the reward heads the trunk outputs)
        rd_run<0, NL, NB>(Rd, a0, ar, ep_lds, lds, ncols, U.bn_s, bn_r, s == 1 ? st_d : nullptr,
                          s < K ? NL : U.rd_trunk_nl);
        if (ok) {
            if (s < K) rn_unstage_l(lds + Rd.out0_off, Rd.out0_kb, NG, U.P, H, t, [&](int f, float v) {
                if constexpr (FUSE) rd_st(hs + (size_t)s * H + f, v); else hs[(size_t)s * H + f] = v;
            });
            rn_unstage_l(lds + trunk, Rd.L[split].in_kb, NG, U.P, H, t, [&](int f, float v) {
                if constexpr (FUSE) rd_st(ts + (size_t)(s - 1) * H + f, v); else ts[(size_t)(s - 1) * H + f] = v;
            });
        }
        if constexpr (FUSE) rd_publish(U, t0, s + 1);                         // h_s (s < K), trunk of step s
    }
}
// TicTacToe resnet_hyper (2 blocks: 10 chain layers, 3x3 board: one column
// block) and Connect4 ResNet-8 (4 blocks: 18 layers, 6x7 board: three)
extern "C" __global__ __launch_bounds__(RD_THREADS) void mz_runroll_chain_r(RUnrollParams U) {
    runroll_chain_r_body<RD_NL, 1>(rn_step(U), blockIdx.x);
}
extern "C" __global__ __launch_bounds__(RD_THREADS) void mz_runroll_chain_r3(RUnrollParams U) {
    runroll_chain_r_body<RD_NL3, 3>(rn_step(U), blockIdx.x);
}

// blockIdx.y = 0: prediction(h_s) for items i = b·KH + s (KH = max(K, 1)):
// step s + 1's value and policy, and step 0's too for s = 0 (Q10: :351 and
// :356 at i = 1 both predict from h_0).  y = 1: the dynamics reward head on
// the trunk output of step s + 1 (items b·K + s): r_{s+1}.
template <bool NARROW, int NBWMAX = 3>
__device__ __forceinline__ void runroll_pred_body(const RUnrollParams& U) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const bool rew = blockIdx.y == 1;
    const RPlan& R = (NARROW ? U.plans_l : U.plans)[rew ? MZ_NET_DYN : MZ_NET_PRED];
    const int NG = NARROW ? U.ng_l : U.ng, H = U.H, A = U.A, K = U.K, K1 = K + 1, KH = K > 0 ? K : 1;
    const int n_items = U.B * KH, t0 = blockIdx.x * NG;
    const int i0 = rew ? U.dyn_split : 0;
    const RnLane t = rn_lane(NG);
    const int it = t0 + t.g;
    const bool ok = it < n_items;
    const size_t ic = (size_t)(ok ? it : 0);
    rn_fill_ktabs(R, lds, NG, U.W, U.P);
    {
        const float* x = (rew ? U.ts : U.hs) + ic * H;
        rn_stage_l(lds + (rew ? R.L[i0].in_off : R.in_off), rew ? R.L[i0].in_kb : R.in_kb, NG, U.P, H, t,
                   [&](int f) { return ok ? x[f] : 0.0f; });
    }
    __syncthreads();
    rn_run<NARROW, true, NBWMAX>(R, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, nullptr, i0);   // :351 / :356, :362
    if (!ok) return;
    const size_t b = ic / KH;
    const int s = (int)(ic - b * KH);
    if (rew) {
        if (t.f0 == 0) U.pr[b * K1 + s + 1] = lds[R.out1_off + t.g];
        return;
    }
    for (int j = s == 0 ? 0 : s + 1; j <= (s + 1 <= K ? s + 1 : 0); ++j) {
        if (t.f0 == 0) U.pv[b * K1 + j] = lds[R.out0_off + t.g];
        float* o = U.pp + (b * K1 + j) * A;
        rn_unstage(lds + R.out1_off, NG, A, t, [&](int f, float v) { o[f] = v; });
    }
}
// mz_runroll_pred_r: runroll_pred_body<true, 1> with the prediction trunk's
// RP_NL layers (1x1 convs of 64 channels on the k-blocked one-item tile) run
// by rd_layer on A fragments loaded at kernel start (all five layers' loads in
// flight together, under the input staging) and epilogue parameters staged in
// LDS; the heads (and the reward-head workgroups, y = 1) on the generic path.
template <int I>
__device__ __forceinline__ void rp_run(const RPlan& R, const float (&ar)[RP_NL][4][4], const float4* ep_lds,
                                       float* lds, int ncols, float bn_s, float bn_r) {
    if constexpr (I < RP_NL) {
        const RLayer L = rn_layer_at(R, I);
        const float (&a1)[1][4][4] = *reinterpret_cast<const float (*)[1][4][4]>(&ar[I]);
        rd_layer<1>(L, a1, ep_lds + I * 64, lds, ncols, bn_s, bn_r);
        __syncthreads();
        rp_run<I + 1>(R, ar, ep_lds, lds, ncols, bn_s, bn_r);
    }
}

// FUSE: an item of mz_runroll_fused_r (ng_l = 1: tile = item b·KH + s), which
// waits until the chain of sample b has published its input; head (prediction
// items): 0 both heads, 1 the value head only, 2 the policy head only (each
// block runs the trunk, then its head: the two heads side by side)
template <bool FUSE>
__device__ __forceinline__ void runroll_pred_r_body(const RUnrollParams& U, bool rew, int tile, int head = 0) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const RPlan& R = U.plans_l[rew ? MZ_NET_DYN : MZ_NET_PRED];
    const int NG = U.ng_l, H = U.H, A = U.A, K = U.K, K1 = K + 1, KH = K > 0 ? K : 1;
    const int n_items = U.B * KH, t0 = tile * NG;
    const int i0 = rew ? U.dyn_split : 0;
    const RnLane t = rn_lane(NG);
    const int it = t0 + t.g;
    const bool ok = it < n_items;
    const size_t ic = (size_t)(ok ? it : 0);
    const int lane = threadIdx.x & 63, ob = threadIdx.x >> 6;
    float4* ep_lds = reinterpret_cast<float4*>(lds + U.rd_ep_off);
    float ar[RP_NL][4][4];
    if (!rew) {
#pragma unroll
        for (int i = 0; i < RP_NL; ++i) rn_load_a(ar[i], U.Wimg, rn_layer_at(R, i), ob, 0, lane);
        for (int i = threadIdx.x; i < RP_NL * 64; i += blockDim.x) {
            const RLayer L = rn_layer_at(R, i >> 6);
            ep_lds[i] = reinterpret_cast<const float4*>(U.Wimg + L.ep_img)[i & 63];
        }
    }
    rn_fill_ktabs(R, lds, NG, U.W, U.P);
    if constexpr (FUSE) {                       // h_s: progress s + 1; trunk of step s + 1: s + 2
        const int bw = (int)(ic / KH), sw = (int)(ic - (size_t)bw * KH);
        rd_wait(U, bw, sw + (rew ? 2 : 1));
    }
    {
        const float* x = (rew ? U.ts : U.hs) + ic * H;
        rn_stage_l(lds + (rew ? R.L[i0].in_off : R.in_off), rew ? R.L[i0].in_kb : R.in_kb, NG, U.P, H, t,
                   [&](int f) { return ok ? (FUSE ? rd_ld(x + f) : x[f]) : 0.0f; });
    }
    __syncthreads();
    if (!rew) {
        rp_run<0>(R, ar, ep_lds, lds, U.P * NG, U.bn_s, 1.0f / U.bn_s);                    // trunk (:351 / :356)
        const int h0 = head == 2 ? RP_NL + U.rp_nv : RP_NL, h1 = head == 1 ? RP_NL + U.rp_nv : -1;
        rn_run<true, true, 1>(R, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, nullptr, h0, h1);   // heads
    } else {
        rn_run<true, true, 1>(R, U.Wimg, U.flat, lds, NG, U.W, U.P, U.bn_s, nullptr, i0);      // :362 reward head
    }
    if (!ok) return;
    const size_t b = ic / KH;
    const int s = (int)(ic - b * KH);
    if (rew) {
        if (t.f0 == 0) U.pr[b * K1 + s + 1] = lds[R.out1_off + t.g];
        return;
    }
    for (int j = s == 0 ? 0 : s + 1; j <= (s + 1 <= K ? s + 1 : 0); ++j) {
        if (head != 2 && t.f0 == 0) U.pv[b * K1 + j] = lds[R.out0_off + t.g];
        float* o = U.pp + (b * K1 + j) * A;
        if (head != 1) rn_unstage(lds + R.out1_off, NG, A, t, [&](int f, float v) { o[f] = v; });
    }
}
extern "C" __global__ __launch_bounds__(RD_THREADS) void mz_runroll_pred_r(RUnrollParams U) {
    runroll_pred_r_body<false>(rn_step(U), blockIdx.y == 1, blockIdx.x);
}

#include "mz_learner_device.h"

// The whole B = small unroll in one launch: blocks [0, n_chain) are the chain
// (representation + K dynamics steps of one sample, mz_runroll_chain_r, and
// with fuse_sample its get_batch draw); the rest are the prediction and
// reward-head items of mz_runroll_pred_r in step-major order, each starting
// as soon as its sample's chain has published the input (rd_wait).  Blocks
// dispatch in index order, so every chain block is resident before any item
// waits on it; the waits are bounded.  Same arithmetic as the two launches.
// Σθ² / ADAM block j of n_l2: slices j, j + n_l2, .. of the 3·MZ_L2_BLOCKS
// (the slice decomposition of mz_learner_grad_kernel, so the same sums)
__device__ __forceinline__ void runroll_l2_block(const RUnrollParams& U, int j) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    double* red = reinterpret_cast<double*>(lds);
    const int tid = threadIdx.x;
    for (int vb0 = 0; vb0 < 3 * MZ_L2_BLOCKS; vb0 += U.n_l2) {        // (block-uniform trip count)
        const int vb = vb0 + j;
        const bool vin = vb < 3 * MZ_L2_BLOCKS;
        const int net = vb / MZ_L2_BLOCKS, blk = vb % MZ_L2_BLOCKS;
        red[tid] = vin ? lg_l2_slice(net, blk, tid, U.netoff, U.flat_w, nullptr, U.ad) : 0.0;
        lg_tree256(red, tid);
        if (tid == 0 && vin)
            __hip_atomic_store(U.part + net * MZ_L2_BLOCKS + blk, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
}

template <int NL, int NB>
__device__ __forceinline__ void runroll_fused_r_body(const RUnrollParams& U, int bi) {
#ifdef MZ_STAMPS   // diagnostic build: per block {start, input published / chain's last publish, end} (s_memrealtime)
    unsigned long long* fs = U.stamps ? U.stamps + 2048 + 4 * bi : nullptr;
    if (fs && threadIdx.x == 0) fs[0] = __builtin_amdgcn_s_memrealtime();
#define RD_FS_END() do { if (fs && threadIdx.x == 0) fs[2] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RD_FS_END() do {} while (0)
#endif
    if (bi < U.n_chain) { runroll_chain_r_body<NL, NB, true>(U, bi); RD_FS_END(); return; }
    if (bi < U.n_chain + U.n_l2) { runroll_l2_block(U, bi - U.n_chain); RD_FS_END(); return; }
    // per step: B value-head items, B policy-head items, B reward heads (K > 0)
    const int ny = U.K > 0 ? 3 : 2, KH = U.K > 0 ? U.K : 1;
    const int idx = bi - U.n_chain - U.n_l2, per_s = ny * U.B;
    const int s = idx / per_s, r = idx - s * per_s, role = r / U.B;
    const int b = r - role * U.B;
    runroll_pred_r_body<true>(U, role == 2, b * KH + s, role == 2 ? 0 : role + 1);
    RD_FS_END();
#undef RD_FS_END
}
// A multi-step launch (U.ms steps, one-dimensional grid): the chain blocks of
// every step first (step-major), so each step's chains are dispatched before
// any item of any step waits on them, then the items step by step
template <int NL, int NB>
__device__ __forceinline__ void runroll_fused_r_entry(const RUnrollParams& U) {
    const int bi = blockIdx.x;
    if (!U.ms) { runroll_fused_r_body<NL, NB>(U, bi); return; }
    const int nc = U.n_chain, per = (U.K > 0 ? 3 : 2) * U.B * (U.K > 0 ? U.K : 1);
    if (bi < U.ms * nc) {
        const int z = bi / nc;
        runroll_fused_r_body<NL, NB>(rn_step(U, z), bi - z * nc);
    } else {
        const int j = bi - U.ms * nc, z = j / per;
        runroll_fused_r_body<NL, NB>(rn_step(U, z), nc + U.n_l2 + (j - z * per));
    }
}
extern "C" __global__ __launch_bounds__(RD_THREADS) void mz_runroll_fused_r(RUnrollParams U) {
    runroll_fused_r_entry<RD_NL, 1>(U);
}
extern "C" __global__ __launch_bounds__(RD_THREADS) void mz_runroll_fused_r3(RUnrollParams U) {
    runroll_fused_r_entry<RD_NL3, 3>(U);
}

// wide tiles of ng items (plans), or one item per workgroup on the narrow
// (chain) plans — B·K workgroups, a short per-layer critical path
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_pred(RUnrollParams U) {
    runroll_pred_body<false>(rn_step(U));
}
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_pred_n(RUnrollParams U) {
    runroll_pred_body<true>(rn_step(U));
}
extern "C" __global__ __launch_bounds__(RN_THREADS) void mz_runroll_pred_n1(RUnrollParams U) {
    runroll_pred_body<true, 1>(rn_step(U));
}
