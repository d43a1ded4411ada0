// mz_small.hip — batched MCTS for SMALL batches (G <= 4 x #CUs): one 512-
// thread workgroup per T in {1, 2, 4} games, so G = 512 spreads over all 256
// CUs of an MI355X instead of the 32 tiles of the 16-game MFMA kernel
// (mz_search.hip), and each simulation waits for the deepest of T games only.
//
// Networks on the VALU.  A stage runs two 64-row "slots", one per 256
// threads (4 waves).  Wave w of a slot owns slot rows 16(w&3)..+15; its four
// 16-lane DPP rows are the four k-quarters q of the canonical dot order
// (mz_dot), lane i of DPP row q is slot row 16(w&3)+i.  Each thread keeps its
// 16 weights W[row][q*kq + j] resident in registers for the whole search and
// loads ONE input element per game, x[q*kq + i]; step j of the 16-step fmaf
// chain takes x[q*kq + j] from lane j of its DPP row as the row_newbcast
// operand of v_fmac_f32_dpp (so the 16 rows of a DPP row must share one input
// vector: the host schedules layers in 16-row groups).  permlane16/32 swaps
// then form ((p0+p1)+(p2+p3)) in every lane, and DPP row 0 adds the bias,
// applies the activation and writes the row.  A dependent fma costs a few
// cycles where a dependent v_mfma_f32_4x4x1 costs 45
// (tools/mfma_rate_probe.hip): the VALU is the latency-optimal unit here.
// Tree (mz_tree_device.h) and hidden states live in LDS; the host builds the
// stage schedule (mz_engine.hip, build_small_schedule).
#include "mz_mlp_device.h"
#include "mz_tree_device.h"

#include "mz_small_params.h"
#include "mz_replay_device.h"
#include "mz_learner_device.h"

#ifdef MZ_STAMPS
#define SM_STAMP(i)                                                              \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            unsigned long long t_ = __builtin_amdgcn_s_memtime();                \
            st_acc[i] += t_ - st_last; st_last = t_;                             \
        }                                                                        \
    } while (0)
// the post-network phase per wave (thread 0: backup, 128: expand, 192: h' store),
// written to the second half of the stamps array (blocks gridDim.x + b)
#define W_STAMP0() unsigned long long w_t0_ = __builtin_amdgcn_s_memtime()
#define W_STAMP(k) do { w_acc[k] += __builtin_amdgcn_s_memtime() - w_t0_; } while (0)
#else
#define SM_STAMP(i) do {} while (0)
#define W_STAMP0() do {} while (0)
#define W_STAMP(k) do {} while (0)
#endif

// Thread -> (slot, slot row, quarter): see the header comment.
__device__ __forceinline__ int sm_slot_row(int tid) {
    return (tid >> 8) * 64 + ((tid >> 6) & 3) * 16 + (tid & 15);   // slot*64 + row
}

// acc += x(lane j of this DPP row) * w, one v_fmac_f32_dpp (fused, IEEE: the
// fmaf of the canonical chain).  Not expressible through the builtins: the
// DPP combiner does not fold into the tied-operand fmac.
template <int J>
__device__ __forceinline__ void fmac_bcast(float& acc, float x, float w) {
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(x), "v"(w), "i"(J));
}

#define SM_F2(j, wj)                                                                              \
    "v_fmac_f32_dpp %0, %2, " wj " row_newbcast:" #j " row_mask:0xf bank_mask:0xf\n\t"            \
    "v_fmac_f32_dpp %1, %3, " wj " row_newbcast:" #j " row_mask:0xf bank_mask:0xf\n\t"

template <int T, int J = 0>
__device__ __forceinline__ void sm_chain(const float (&w)[16], const float (&x)[T], float (&acc)[T]) {
    if constexpr (T == 2 && J == 0) {
        // the two games' chains interleaved in one block.  The DPP hazard (a
        // VALU write followed by a DPP read, 2 wait states) concerns the
        // lane-swizzled source x, which nothing writes inside the chain; the
        // compiler also pads for the accumulator (an s_nop per pair), which
        // the interleave already separates by one instruction.  One s_nop 1
        // up front covers x written by VALU just before (the fused first stage).
        asm volatile("s_nop 1\n\t"
                     SM_F2(0, "%4") SM_F2(1, "%5") SM_F2(2, "%6") SM_F2(3, "%7")
                     SM_F2(4, "%8") SM_F2(5, "%9") SM_F2(6, "%10") SM_F2(7, "%11")
                     SM_F2(8, "%12") SM_F2(9, "%13") SM_F2(10, "%14") SM_F2(11, "%15")
                     SM_F2(12, "%16") SM_F2(13, "%17") SM_F2(14, "%18") SM_F2(15, "%19")
                     : "+v"(acc[0]), "+v"(acc[1])
                     : "v"(x[0]), "v"(x[1]), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]),
                       "v"(w[6]), "v"(w[7]), "v"(w[8]), "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]),
                       "v"(w[14]), "v"(w[15]));
    } else if constexpr (J < 16) {
#pragma unroll
        for (int g = 0; g < T; ++g) fmac_bcast<J>(acc[g], x[g], w[J]);
        sm_chain<T, J + 1>(w, x, acc);
    }
}

// The search's first stage reads its inputs straight from the hidden-state
// store (no gather copy, no barrier): prediction's input x_pred = the parent's
// h, dynamics' x_dyn = 2h ⊕ a/|A| (make_state_action, SelfPlay.jl:7-14; Q1's
// in-place doubling of the parent is written back after the networks).
// The learner's steps use the same fusion (FI = 2): x_pred = h_{i-1} read
// from the activation buffer (h_out, [k][T]) and x_dyn = 2h ⊕ a_{i-1}/|A|
// (make_dynamics_input, Learning.jl:293-304): `hid` = act + h_out, `aval` =
// the step's a/|A| of game 0 (game g's at aval[g * NN]).
struct SmFusedIn {
    const float* hid; const int* leaf_e; const int* leaf_a; const float* aval;
    int NN, H, plane, x_pred, x_dyn;
};

// This thread's input offset in a stage with record R: x[q*kq + i] of the T
// games (rows beyond kq meet zero weights; the 64-row input buffers are zero
// beyond K, so every step is exact); q·kq as a 24-bit multiply (full rate,
// where a 32-bit one is quarter rate)
template <int T>
__device__ __forceinline__ int sm_xoff(int4 R) {      // (in bytes)
    const int q = (threadIdx.x >> 4) & 3, i = threadIdx.x & 15;
    return (R.x + ((int)__umul24((unsigned)q, (unsigned)R.y) + i) * T) * 4;
}

// One stage.  R = this thread's record of stage K, xo its input offset
// (sm_xoff); the record of stage K+1 (constant for the whole kernel) is
// fetched while stage K computes, and its offset formed before the barrier,
// so the next stage's input load issues right after it (xo is updated).
// BNM: 1 = the record's BatchNorm bit is tested (make_dense with BatchNorm, test mode), 0 = the
// nets have no BatchNorm layer (the search kernels' plain instances: no test, no (γ, β) load)
template <int T, int FI = 0, int BNM = 1>
__device__ __forceinline__ int4 sm_stage(const float (&w)[16], int4 R, int& xo, const int4* rec_next, float* lds,
                                         const SmFusedIn* fi = nullptr, const float2* bnp = nullptr) {
    const int q = (threadIdx.x >> 4) & 3;
    const float* xp = reinterpret_cast<const float*>(reinterpret_cast<const char*>(lds) + xo);
    float x[T];
    if constexpr (FI != 0) {
        const int k = (int)__umul24((unsigned)q, (unsigned)R.y) + (int)(threadIdx.x & 15);
        const bool pred = R.x == fi->x_pred, dyn = R.x == fi->x_dyn;
#pragma unroll
        for (int g = 0; g < T; ++g) {
            float hv, av;
            if constexpr (FI == 1) {
                const float* hp = fi->hid + ((size_t)g * fi->NN + fi->leaf_e[g]) * fi->H;
                hv = k < fi->H ? hp[k] : 0.0f;
                av = fi->aval[fi->leaf_a[g]];
            } else {
                hv = k < fi->H ? fi->hid[k * T + g] : 0.0f;
                av = fi->aval[g * fi->NN];
            }
            x[g] = pred ? hv : dyn ? (k < fi->H ? hv * 2.0f : k < fi->H + fi->plane ? av : 0.0f) : xp[g];
        }
    } else if constexpr (T == 1) {
        x[0] = xp[0];
    } else if constexpr (T == 2) {
        const float2 v = *reinterpret_cast<const float2*>(xp);
        x[0] = v.x; x[1] = v.y;
    } else {
        const float4 v = *reinterpret_cast<const float4*>(xp);
        x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
    }
    const int4 Rn = *rec_next;
    float acc[T];
#pragma unroll
    for (int g = 0; g < T; ++g) acc[g] = 0.0f;
    sm_chain<T>(w, x, acc);
    // ((p0+p1)+(p2+p3)) in every lane: with both operands equal, the two
    // halves of a permlane swap are {own, partner} in row order, so their sum
    // is p_even + p_odd in both rows of each pair
#pragma unroll
    for (int g = 0; g < T; ++g) {
        const auto s1 = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, acc[g]),
                                                         __builtin_bit_cast(unsigned, acc[g]), false, false);
        const float t = __builtin_bit_cast(float, (unsigned)s1[0]) + __builtin_bit_cast(float, (unsigned)s1[1]);
        const auto s2 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, t),
                                                         __builtin_bit_cast(unsigned, t), false, false);
        acc[g] = __builtin_bit_cast(float, (unsigned)s2[0]) + __builtin_bit_cast(float, (unsigned)s2[1]);
    }
    // every DPP row now holds the T sums: DPP row q < T writes game q's row,
    // so the T epilogues run side by side on different lanes
    if (q < T && R.z >= 0) {
        float v = acc[0];
#pragma unroll
        for (int g = 1; g < T; ++g) v = q == g ? acc[g] : v;
        const int o = R.z & 0x1fffffff;
        float d = v + __int_as_float(R.w);
        if constexpr (BNM != 0)
            if ((R.z >> 29) & 1) { const float2 gb = *bnp; d = mz_bn_apply(d, gb.x, gb.y); }
        lds[o + q] = (R.z >> 30) != 0 ? mz_relu(d) : d;
    }
    xo = sm_xoff<T>(Rn);
    asm volatile("" : "+v"(xo));     // formed here, not sunk below the barrier
    __syncthreads();
    return Rn;
}

// rec: this thread's record of stage 0 ([stage][slot][row] int4, stride 128)
template <int T, int NMAX, int FI, int OFF, int BNM, int K = 0>
__device__ __forceinline__ void sm_run_k(int n, const float (&wr)[NMAX][16], int4 R, int xo, const int4* rec,
                                         float* lds, const SmFusedIn* fi, const float2* bnp) {
    if constexpr (K + OFF < NMAX) {
        if (K < n) {
            const float2* bk = bnp + K * (SM_SLOTS * 64);
            const int4 Rn = K == 0 && FI != 0
                ? sm_stage<T, FI, BNM>(wr[K + OFF], R, xo, rec + (K + 1) * (SM_SLOTS * 64), lds, fi, bk)
                : sm_stage<T, 0, BNM>(wr[K + OFF], R, xo, rec + (K + 1) * (SM_SLOTS * 64), lds, nullptr, bk);
            sm_run_k<T, NMAX, FI, OFF, BNM, K + 1>(n, wr, Rn, xo, rec, lds, fi, bnp);
        }
    }
}

// FI: 0 = inputs from the activation buffer, 1 = the search's fused first
// stage, 2 = the learner's (SmFusedIn).  Stage K runs on register set K + OFF.
// bnp: this thread's (γ, β) column, laid out as `rec` (read only by BatchNorm rows).
template <int T, int NMAX, int FI = 0, int OFF = 0, int BNM = 1>
__device__ __forceinline__ void sm_run(int n, const float (&wr)[NMAX][16], const int4* rec, float* lds,
                                       const SmFusedIn* fi, const float2* bnp) {
    const int4 R0 = rec[0];
    sm_run_k<T, NMAX, FI, OFF, BNM>(n, wr, R0, sm_xoff<T>(R0), rec, lds, fi, bnp);
}

// Weights of this thread's (slot, row, quarter) for stages 0..n-1 from the
// host image (sm_widx: chunk i of the slot's 256 threads is 4 KiB contiguous).
// Stages [k0, k1) only (others untouched: sm_run never reads stages >= n,
// so the representation's free registers can be filled with sim stages
// while it runs).
template <int NMAX, int DST = 0>   // image stage k -> register set k + DST
__device__ __forceinline__ void sm_load(int k0, int k1, const float* W, float (&wr)[NMAX][16], const uint32_t* nzm,
                                        const float4* zero16) {
    const int tid = threadIdx.x, sl = tid >> 8, t = tid & 255, q = (tid >> 4) & 3;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t mk[NMAX - DST];                           // the wave's masks: one batch of scalar loads
#pragma unroll
    for (int k = 0; k < NMAX - DST; ++k) mk[k] = nzm[w * SM_NZM_ST + k];
#pragma unroll
    for (int k = 0; k < NMAX - DST; ++k) {
        if (k >= k0 && k < k1) {
            const float4* src = reinterpret_cast<const float4*>(W + (((size_t)k * SM_SLOTS + sl) * 4) * 1024) + t;
            const uint32_t m = mk[k] >> (4 * q);       // this DPP row's chunks
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // a skipped chunk reads the shared zero line (branch-free; one
                // cache line for every skipping lane)
#ifdef MZ_NO_WLOAD   // diagnostic only (wrong results): the setup without the weight stream
                const float4 v = make_float4((float)(m >> i & 1u), 0.0f, 0.0f, 0.0f);
#else
                const float4 v = *((m >> i) & 1u ? src + i * 256 : zero16);
#endif
                wr[k + DST][4 * i] = v.x; wr[k + DST][4 * i + 1] = v.y; wr[k + DST][4 * i + 2] = v.z;
                wr[k + DST][4 * i + 3] = v.w;
            }
        }
    }
}

template <int T, int BNM>
__device__ __forceinline__ void small_body(const SmallParams& P) {
#ifdef MZ_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
    unsigned long long w_acc[3] = {0, 0, 0};
#endif
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int A = P.A, S = P.S, H = P.H;
    const int E = (S + 1) * A, NN = S + 1;
    const int PS = 2 * (S + 2);
    const int nrec = P.n_sim + P.n_root;
    float* act = smem;                                           // act_total floats (multiple of 4)
    int* rec = reinterpret_cast<int*>(act + P.act_total);        // [nrec][SM_REC_INTS]
    float* hid = reinterpret_cast<float*>(rec + (nrec + 1) * SM_REC_INTS);   // [T][S+1][H] (+1: look-ahead slack)
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
    // si + 224 .. 231: unused (formerly the leaf value / reward read-outs)
    float* sg_noise = reinterpret_cast<float*>(si + 232);       // [4][16] root exploration noise
    int* sg_path = si + 296;                                      // [T][2(S+2)]
    // select / gather tables in LDS (they sit on the per-level critical path)
    double* l_pbc = reinterpret_cast<double*>(si + 296 + (T * PS + 3) / 4 * 4);   // [S+2]
    double* l_sqrt = l_pbc + (S + 2);                                           // [S+2]
    float* l_aval = reinterpret_cast<float*>(l_sqrt + (S + 2));                 // [32]
    double* l_pbterm = reinterpret_cast<double*>(l_aval + MZ_MAX_ACTIONS);     // [pbterm_count(S)]
    char* lds_tree = reinterpret_cast<char*>(l_pbterm + pbterm_count(S));
    // the cached select (mz_tree_device.h select_path_cached): per game the
    // entries [NN], the last path's (slot, N) per level [S+2], N per slot [NN]
    uint2* c_cache = reinterpret_cast<uint2*>(lds_tree + (size_t)T * P.tree_game_bytes);
    uint2* c_lvl = c_cache + T * NN;
    int* c_nN = reinterpret_cast<int*>(c_lvl + T * (S + 2));
    // per game, written by backup for the recompute: {min / max moved (recompute
    // every node), select depth, tag, root legal mask} and {min, max}
    int4* c_hdr = reinterpret_cast<int4*>(reinterpret_cast<char*>(smem) +                 // [4], 16-byte aligned
                                          ((reinterpret_cast<char*>(c_nN + T * NN) - reinterpret_cast<char*>(smem) + 15) & ~15));
    float2* c_mmx = reinterpret_cast<float2*>(c_hdr + 4);         // [4]
    // [4] per game: the select's start level (the last path's prefix the
    // recompute found unchanged; 0 = from the root)
    int* c_skip = reinterpret_cast<int*>(c_mmx + 4);
    float2* bnl = reinterpret_cast<float2*>(c_skip + 4);          // [nrec][slot][64] BatchNorm (γ, β) (P.bn)

    const int tid = threadIdx.x;
    const int g = tid >> 4, a = tid & 15, lane = tid & 63;
    const int tile0 = blockIdx.x * T;
    const bool tree_thread = tid < 16 * T;
    const int gg = tile0 + g;
    const bool active = tree_thread && gg < P.G;
    const uint32_t gid = P.game_offset + (uint32_t)gg;
    int* path = sg_path + (tree_thread ? g : 0) * PS;
    TreeView tree = tree_view(lds_tree + (size_t)(tree_thread ? g : 0) * P.tree_game_bytes, E, NN);
    // this thread's (slot, row) record column; one extra stage of slack is
    // read (never used) past each schedule's last stage
    const int4* rec_sim = reinterpret_cast<const int4*>(rec) + sm_slot_row(tid);
    const int4* rec_root = rec_sim + P.n_sim * (SM_SLOTS * 64);
    const float2* bn_sim = bnl + sm_slot_row(tid);
    const float2* bn_root = bn_sim + P.n_sim * (SM_SLOTS * 64);

    // ---- weight-image loads first: in flight under the setup copies.  The
    // representation (SelfPlay.jl:234) runs on its own schedule; the sim
    // stages it leaves free are preloaded, the rest reloaded after it.
    float wr[SM_MAX_SIM][16];
    sm_load<SM_MAX_SIM>(0, P.n_root, P.w_root, wr, P.nzm + P.n_sim, P.zero16);
    sm_load<SM_MAX_SIM>(P.n_root, P.n_sim, P.w_sim, wr, P.nzm, P.zero16);
    for (int i = tid; i < P.act_total; i += SM_THREADS) act[i] = 0.0f;
    for (int i = tid; i < S + 2; i += SM_THREADS) { l_pbc[i] = P.pbc_tab[i]; l_sqrt[i] = P.sqrt_tab[i]; }
    if (tid < A) l_aval[tid] = P.aval_tab[tid];
    for (int i = tid; i < (int)pbterm_count(S); i += SM_THREADS) l_pbterm[i] = P.pbterm[i];
    for (int i = tid; i < nrec * SM_REC_INTS; i += SM_THREADS) rec[i] = P.rec[i];
    __syncthreads();
    for (int i = tid; i < nrec * SM_SLOTS * 64; i += SM_THREADS)
        rec[4 * i + 3] = __float_as_int(P.bias[i]);
    if (P.bn)
        for (int i = tid; i < nrec * SM_SLOTS * 64; i += SM_THREADS)
            bnl[i] = make_float2(P.bias[nrec * SM_SLOTS * 64 + i], P.bias[2 * nrec * SM_SLOTS * 64 + i]);
    // ---- root inputs
    for (int i = tid; i < T * P.obs_feat; i += SM_THREADS) {
        const int gl = i / P.obs_feat, k = i - gl * P.obs_feat;
        const int ggl = tile0 + gl;
        act[P.x_rep + k * T + gl] = ggl < P.G ? P.obs[(size_t)ggl * P.obs_feat + k] : 0.0f;
    }
    for (int i = tid; i < T * NN; i += SM_THREADS) c_cache[i] = make_uint2(0u, 0u);
    if (tid < 4) { c_hdr[tid] = make_int4(0, -1, 1, 0); c_mmx[tid] = make_float2(0.0f, 0.0f); c_skip[tid] = 0; }
    int ver = 1;                                                  // wave 0: the tag of this lane's game
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

    // the root's exploration noise depends only on the legal set: drawn here,
    // lane-parallel, while the weight loads are in flight
    if (P.exploration && active)
        sg_noise[16 * g + a] = root_noise_lane(sg_legal[g], a, A, P.seed, gid, P.rng_step, P.dirichlet_alpha,
                                               sg_stage + 16 * g);
    sm_run<T, SM_MAX_SIM, 0, 0, BNM>(P.n_root, wr, rec_root, act, nullptr, bn_root);
    for (int i = tid; i < T * H; i += SM_THREADS) {     // h -> hidden slot 0 and the prediction input
        const int gl = i / H, k = i - gl * H;
        const float h = act[P.h_out + k * T + gl];
        hid[(size_t)gl * NN * H + k] = h;
        act[P.x_pred + k * T + gl] = h;
    }
    // prediction ‖ dynamics weights: resident for the whole search
    sm_load<SM_MAX_SIM>(0, P.n_root < P.n_sim ? P.n_root : P.n_sim, P.w_sim, wr, P.nzm, P.zero16);
    __syncthreads();
    // prediction(h) for the root (:239); the dynamics half runs on zeros, unused
    sm_run<T, SM_MAX_SIM, 0, 0, BNM>(P.n_sim, wr, rec_sim, act, nullptr, bn_sim);

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
    if (P.exploration && active && a < A && ((legal >> a) & 1u))     // add_exploration_noise! (:102-109)
        tree.p(a) = tree.p(a) * (1.0f - P.exploration_eps) + sg_noise[16 * g + a] * P.exploration_eps;
    __syncthreads();
    SM_STAMP(0);

    const SmFusedIn fin{hid, sg_leaf_e, sg_leaf_a, l_aval, NN, H, P.plane, P.x_pred, P.x_dyn};
    // Per simulation, three workgroup barriers besides the 8 network stages:
    // wave 0 owns the trees (T <= 4 games x 16 lanes), so select -> gather and
    // backup -> next select need only wave-local ordering.
    for (int s = 0; s < S; ++s) {
        if (tid < 64) {
            // ---- select (:256-268)
            if (active) {
                // the start level and its node / incoming edge from the last path
#ifdef MZ_NO_SKIP   // A/B: every walk from the root
                const int D = 0;
#else
                const int D = c_skip[g];
#endif
                const int e0 = D > 0 ? path[2 * D + 1] : 0;
                const uint32_t npc0 = D > 0 ? tree.nc(path[2 * D]) : 0u;
                const SelectOut so = select_path_cached(tree, c_cache + g * NN, (uint32_t)ver, path, sg_rootN[g],
                                                        sg_root_tp[g], legal, sg_mmin[g], sg_mmax[g], a, lane, A,
                                                        P.players, l_pbterm, P.seed, gid, P.rng_step, s, nullptr,
                                                        nullptr, D, e0, npc0);
                if (a == 0) { sg_leaf_e[g] = so.leaf_e; sg_leaf_a[g] = so.leaf_a; sg_vtp[g] = so.vtp; sg_depth[g] = so.depth; }
            }
            __builtin_amdgcn_wave_barrier();
            SM_STAMP(1);
#ifdef MZ_STAMPS
            if (threadIdx.x == 0) {             // slot 7: select levels walked (max over the T games)
                int md = 0;
                for (int gl = 0; gl < T; ++gl) md = md > sg_depth[gl] ? md : sg_depth[gl];
                st_acc[7] += (unsigned long long)md;
            }
#endif
        }
        __syncthreads();
        SM_STAMP(2);
        // ---- prediction(parent.h) ‖ dynamics(2h ⊕ a/|A|): the first stage
        // reads the parent's h from the hidden-state store (gather fused)
        sm_run<T, SM_MAX_SIM, 1, 0, BNM>(P.n_sim, wr, rec_sim, act, &fin, bn_sim);
        SM_STAMP(3);
        const int e_new = s + 1;
        // expand (wave 2) runs beside the read-outs + backup (wave 0): they
        // touch disjoint LDS — the new slot's edges vs the path edges, the
        // leaf edge's child link and the new slot's reward / to_play
        if (tid < 64) {
            // ---- value / reward read-out activations, then backpropagate! (:190-217)
            if (active) {
                // the backup's loads first (two players): in flight under the read-outs
                const int tl = sg_vtp[g];
                const int depth = sg_depth[g];
                const BackupPre bpre = backup_preload(tree, path, depth, a);
                // one activation per lane (even lanes the value, odd the reward, both
                // f64 tanh chains run at once), then each quad's lanes 0 / 1 to all
                // four by DPP quad_perm [0,0,0,0] / [1,1,1,1]
                const bool odd = (a & 1) != 0;
#ifdef MZ_DIAG_TANH_TWICE     // diagnostic (same results): the read-out activations twice
                float rin = act[(odd ? P.r_out : P.v_out) + g];
                const float ro0 = mz_post_act(odd ? P.r_act : P.v_act, rin);
                asm volatile("" : "+v"(rin) : "v"(ro0));
                const float ro = mz_post_act(odd ? P.r_act : P.v_act, rin);
#else
                const float ro = mz_post_act(odd ? P.r_act : P.v_act, act[(odd ? P.r_out : P.v_out) + g]);
#endif
                const float val = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                    0, __builtin_bit_cast(int, ro), 0x00, 0xF, 0xF, false));
                const float rew = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                    0, __builtin_bit_cast(int, ro), 0x55, 0xF, 0xF, false));
#ifdef MZ_STAMPS
                if (threadIdx.x == 0) asm volatile("" :: "v"(val), "v"(rew));
#endif
                SM_STAMP(5);                    // stamp build: slot 5 = the read-out activations
                W_STAMP0();
                if (a == 0) {
                    const int li = sg_leaf_e[g] * A + sg_leaf_a[g];
                    tree.nc(li) = (tree.nc(li) & 0xffffu) | ((uint32_t)(e_new + 1) << 16);
                    tree.nr[e_new] = rew;
                    tree.ntp[e_new] = (int8_t)tl;
                    path[2 * depth + 1] = e_new;
                }
                __builtin_amdgcn_wave_barrier();
                int rN = sg_rootN[g];
                float rW = sg_rootW[g], mmin = sg_mmin[g], mmax = sg_mmax[g];
                const uint32_t omin = __float_as_uint(mmin), omax = __float_as_uint(mmax);
                if (P.players == 2)
                    backup_path_pre(tree, path, bpre, depth, val, rew, e_new, tl, P.discount, rN, rW, sg_root_tp[g],
                                    mmin, mmax, a, c_lvl + g * (S + 2), c_nN + g * NN);
                else
                    backup_path(tree, path, depth, val, tl, A, P.players, P.discount, rN, rW, sg_root_tp[g], mmin,
                                mmax, a, c_lvl + g * (S + 2), c_nN + g * NN);
                const bool moved = __float_as_uint(mmin) != omin || __float_as_uint(mmax) != omax;
                ver += moved ? 1 : 0;                     // min / max moved: every entry is stale
                if (a == 0) {
                    sg_rootN[g] = rN; sg_rootW[g] = rW; sg_mmin[g] = mmin; sg_mmax[g] = mmax;
                    c_hdr[g] = make_int4(moved ? 1 : 0, depth, ver, (int)legal);
                    c_mmx[g] = make_float2(mmin, mmax);
                    c_skip[g] = moved ? 0 : depth;            // lowered by the recompute's path rows
                }
                W_STAMP(0);
            }
        } else if (tid >= 128 && tid < 128 + 16 * T) {
            W_STAMP0();
            // ---- expand slot s+1 (:280): wave 2 lanes 16 g2 + a2 (g2, a2 as wave 0's g, a)
            const int g2 = (tid - 128) >> 4;
            const bool active2 = tile0 + g2 < P.G;
            TreeView tree2 = tree_view(lds_tree + (size_t)g2 * P.tree_game_bytes, E, NN);
#ifdef MZ_DIAG_EXPAND_TWICE   // diagnostic (same results): the double softmax twice — is expand on the critical path?
            float lgt = act[P.p_out + a * T + g2];
            const float prior0 = double_softmax_prior(a < A ? lgt : 0.0f, a, A, sg_legal[g2], sg_stage + 16 * g2);
            asm volatile("" : "+v"(lgt) : "v"(prior0));
            const float prior = double_softmax_prior(a < A ? lgt : 0.0f, a, A, sg_legal[g2], sg_stage + 16 * g2);
#else
            const float prior = double_softmax_prior(a < A ? act[P.p_out + a * T + g2] : 0.0f, a, A, sg_legal[g2],
                                                     sg_stage + 16 * g2);
#endif
            if (active2) init_edges(tree2, e_new, a, A, prior);
            W_STAMP(1);
        } else if (tid >= 192) {
            W_STAMP0();
            for (int i = tid - 192; i < T * H; i += SM_THREADS - 192) {   // store h'; parent h *= 2 (Q1)
                const int gl = i / H, k = i - gl * H;
                hid[((size_t)gl * NN + e_new) * H + k] = act[P.h_out + k * T + gl];
                if (tile0 + gl < P.G) {
                    float* hp = hid + ((size_t)gl * NN + sg_leaf_e[gl]) * H + k;
                    *hp = *hp * 2.0f;
                }
            }
            W_STAMP(2);
        }
        __syncthreads();
        SM_STAMP(4);
        // ---- the cached select's entries for the next simulation (all waves,
        // one 16-lane row per node): the nodes of this path, or every
        // expanded node when min / max moved
        if (s + 1 < S) {
            const int r = tid >> 4, gq = r % T, j0 = r / T;
            // every read of the first row is independent of the others: the header,
            // min / max, and both candidate (slot, N) sources
            int4 hd = c_hdr[gq];
            float2 mm = c_mmx[gq];
            uint2 l0 = c_lvl[gq * (S + 2) + j0];
            int n0 = c_nN[gq * NN + j0];
            asm volatile("" : "+v"(hd.x), "+v"(hd.y), "+v"(hd.z), "+v"(hd.w), "+v"(mm.x), "+v"(mm.y), "+v"(l0.x),
                              "+v"(l0.y), "+v"(n0));   // all issued together, one wait
            const bool full = hd.x != 0;
            const int n = full ? s + 2 : hd.y + 1;
            const bool lgl = a < A && (((uint32_t)hd.w >> a) & 1u);
            const TreeView tq = tree_view(lds_tree + (size_t)gq * P.tree_game_bytes, E, NN);
            uint2* cq = c_cache + gq * NN;
            // a path row whose new choice leaves the last path (or ties) bounds the
            // next select's skip-ahead: levels below it are retraced as they were
            const int* pq = sg_path + gq * PS;
            const int pe0 = !full && j0 < hd.y ? pq[2 * (j0 + 1)] : 0;
            if (j0 < n) {
                const int ch = cache_row(tq, cq, (uint32_t)hd.z, full ? j0 : (int)l0.x, full ? n0 : (int)l0.y, lgl,
                                         a, A, mm.x, mm.y, l_pbterm, lane);
                if (!full && a == 0 && (j0 >= hd.y || ch != pe0 - (int)l0.x * A)) atomicMin(c_skip + gq, j0);
            }
            for (int j = j0 + SM_THREADS / 16 / T; j < n; j += SM_THREADS / 16 / T) {   // deep paths, large trees
                int slot, Np;
                if (full) { slot = j; Np = c_nN[gq * NN + j]; }
                else { const uint2 l = c_lvl[gq * (S + 2) + j]; slot = (int)l.x; Np = (int)l.y; }
                const int ch = cache_row(tq, cq, (uint32_t)hd.z, slot, Np, lgl, a, A, mm.x, mm.y, l_pbterm, lane);
                if (!full && a == 0 && (j >= hd.y || ch != pq[2 * (j + 1)] - slot * A)) atomicMin(c_skip + gq, j);
            }
            __syncthreads();
            SM_STAMP(6);                           // stamp build: slot 6 = the cache recompute (+ finish)
        }
    }
    __syncthreads();

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
        if (P.dump_tree) {
            TreeView dst = tree_view(P.tree + (size_t)gg * P.tree_game_bytes, E, NN);
            dump_tree(tree, dst, E, NN, a);
        }
    }
#ifdef MZ_STAMPS
    SM_STAMP(6);
    if (threadIdx.x == 0 && P.stamps)
        for (int i = 0; i < 8; ++i) P.stamps[blockIdx.x * 8 + i] = st_acc[i];
    if (P.stamps && (threadIdx.x == 0 || threadIdx.x == 128 || threadIdx.x == 192)) {
        const int k = threadIdx.x == 0 ? 0 : threadIdx.x == 128 ? 1 : 2;
        P.stamps[(gridDim.x + blockIdx.x) * 8 + k] = w_acc[k];
    }
#endif
}

// (the _bn instances: nets with BatchNorm FC layers, SmallParams.bn)
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small1(SmallParams P) { small_body<1, 0>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small2(SmallParams P) { small_body<2, 0>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small4(SmallParams P) { small_body<4, 0>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small1_bn(SmallParams P) { small_body<1, 1>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small2_bn(SmallParams P) { small_body<2, 1>(P); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_search_small4_bn(SmallParams P) { small_body<4, 1>(P); }

// ---------------------------------------------------------------- learner
// K-step unroll of Learning.jl:327-343 (Q10 alignment, as mz_unroll_kernel):
// h0 = representation(obs); for i = 1..K: prediction(h_{i-1}) ‖
// dynamics(2h_{i-1} ⊕ a_{i-1}/|A|) on the search's stage schedule.  Stored:
// pv/pp at i (and at 0 for i = 1) = prediction of h_{i-1}; pr at i = reward
// of step i, pr at 0 = 0.  Policy = softmax of the logits in the oracle's
// order; value / reward with their read-out activations — applied by the
// loss kernel, which visits every (sample, step) pair in parallel.
// The per-call arrays of one unroll: the batch, the raw read-outs and the
// weight image (the one-step kernels pass P's own, sm_io; the multi-step
// kernel its step's batch set and bank image)
struct SmIO {
    const float* obs; const float* actions; float* pv; float* pp; float* pr;
    const float* w_sim; const float* w_root; const float* bias;
};
__device__ __forceinline__ SmIO sm_io(const SmallUnrollParams& P) {
    return SmIO{P.obs, P.actions, P.pv, P.pp, P.pr, P.w_sim, P.w_root, P.bias};
}

template <int T, int BNM>
__device__ __forceinline__ void unroll_body(const SmallUnrollParams& P, int lb, const SmIO& io) {
#ifdef MZ_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int K = P.K, A = P.A, H = P.H;
    const int nrec = P.n_sim + P.n_root;
    float* act = smem;
    int* rec = reinterpret_cast<int*>(act + P.act_total);
    float* aval = reinterpret_cast<float*>(rec + (nrec + 1) * SM_REC_INTS);    // [T][K+1] a/|A| per step
    float2* bnl = reinterpret_cast<float2*>(aval + 64);                     // [nrec][slot][64] (γ, β) (P.bn)
    const int tid = threadIdx.x;
    const int tile0 = lb * T;
    // per-thread item of the per-step loops (each has < SM_THREADS items)
    const int o_gl = tid / (A + 2), o_c = tid - o_gl * (A + 2);      // raw outputs: tid < T*(A+2)
    // Every global load of the setup is issued before the weight image (a
    // wave's loads complete in order, vmcnt): the prefetch header, the stage
    // records with their biases merged, the batch's observation and actions.
    // Without a prefetch the sampler (waves 0..T-1) runs first and the batch is
    // read after it.  The chain is then one global round trip, not three.
    const int nri = nrec * SM_SLOTS * 64;                             // int4 records (one per slot row)
    constexpr int RPT = ((SM_MAX_SIM + SM_MAX_ROOT) * SM_SLOTS * 64 + SM_THREADS - 1) / SM_THREADS;
    const bool sample_first = !P.pf_hdr && P.sample;
    if (sample_first && (tid >> 6) < T && tile0 + (tid >> 6) < P.B) rp_sample_one(P.rp, tile0 + (tid >> 6), tid & 63);
    if (sample_first) { __threadfence_block(); __syncthreads(); }
    long long hd[4] = {0, 0, 0, 0}, cnt0 = 0;
    if (P.pf_hdr) { hd[0] = P.pf_hdr[0]; hd[1] = P.pf_hdr[1]; hd[2] = P.pf_hdr[2]; hd[3] = P.pf_hdr[3]; cnt0 = P.rp.counters[0]; }
    int rx[RPT], ry[RPT], rz[RPT];                                    // (plain ints: the HIP vector type
    float bv[RPT];                                                    //  kept the array in scratch)
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int i = tid + u * SM_THREADS;
        const int ic = i < nri ? i : 0;
        const int4 r = reinterpret_cast<const int4*>(P.rec)[ic];
        rx[u] = r.x; ry[u] = r.y; rz[u] = r.z;
        bv[u] = io.bias[ic];
    }
    const int o_i = tid / P.obs_feat, o_k = tid - o_i * P.obs_feat;   // observation item: tid < T*obs_feat
    const int a_i = tid / (K + 1), a_k = tid - a_i * (K + 1);        // action item: tid < T*(K+1)
    const bool o_in = tid < T * P.obs_feat && tile0 + o_i < P.B, a_in = tid < T * (K + 1) && tile0 + a_i < P.B;
    float ov = o_in ? io.obs[(size_t)(tile0 + o_i) * P.obs_feat + o_k] : 0.0f;
    float av = a_in ? io.actions[(size_t)(tile0 + a_i) * (K + 1) + a_k] : 0.0f;
    float wr[SM_MAX_SIM][16];
    // the representation runs on register sets RO.. (RO + n_root), so the first
    // RO sim stages are loaded now and step 1 starts on them while the sets
    // the representation used are reloaded (no exposed reload)
    constexpr int RO = SM_MAX_SIM - SM_MAX_ROOT;
    sm_load<SM_MAX_SIM, RO>(0, P.n_root, io.w_root, wr, P.nzm + P.n_sim, P.zero16);
    sm_load<SM_MAX_SIM>(0, RO < P.n_sim ? RO : P.n_sim, io.w_sim, wr, P.nzm, P.zero16);
    sm_load<SM_MAX_SIM>(RO + P.n_root, P.n_sim, io.w_sim, wr, P.nzm, P.zero16);
    // a prefetched batch (the previous launch sampled this step's) is used
    // while its header still matches the shard; otherwise (the first step after
    // the shard changed) waves 0..T-1 sample in place and the batch is re-read
    const bool have = P.pf_hdr && hd[0] == P.pf_epoch && hd[1] == cnt0 && hd[2] == (long long)P.rp.step &&
                      hd[3] == (long long)P.B;
    if (P.pf_hdr && P.sample && !have) {
        if ((tid >> 6) < T && tile0 + (tid >> 6) < P.B) rp_sample_one(P.rp, tile0 + (tid >> 6), tid & 63);
        __threadfence_block();
        __syncthreads();
        ov = o_in ? io.obs[(size_t)(tile0 + o_i) * P.obs_feat + o_k] : 0.0f;
        av = a_in ? io.actions[(size_t)(tile0 + a_i) * (K + 1) + a_k] : 0.0f;
    }
    for (int i = tid; i < P.act_total; i += SM_THREADS) act[i] = 0.0f;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int i = tid + u * SM_THREADS;
        if (i < nri) reinterpret_cast<int4*>(rec)[i] = make_int4(rx[u], ry[u], rz[u], __float_as_int(bv[u]));
    }
    if (tid < SM_REC_INTS / 4) reinterpret_cast<int4*>(rec)[nri + tid] = make_int4(0, 0, -1, 0);   // slack stage
    if (P.bn)
        for (int i = tid; i < nri; i += SM_THREADS) bnl[i] = make_float2(io.bias[nri + i], io.bias[2 * nri + i]);
    __syncthreads();                               // act zeroed before the inputs land in it
    if (o_in) act[P.x_rep + o_k * T + o_i] = ov;
    if (a_in) aval[a_i * (K + 1) + a_k] = av / (float)A;           // make_dynamics_input's a/|A| (:294)
    __syncthreads();
    SM_STAMP(0);                                   // setup: records, bias gather, inputs
    const int4* rec_sim = reinterpret_cast<const int4*>(rec) + sm_slot_row(tid);
    const int4* rec_root = rec_sim + P.n_sim * (SM_SLOTS * 64);
    const float2* bn_sim = bnl + sm_slot_row(tid);
    const float2* bn_root = bn_sim + P.n_sim * (SM_SLOTS * 64);
    sm_run<T, SM_MAX_SIM, 0, RO, BNM>(P.n_root, wr, rec_root, act, nullptr, bn_root);
    SM_STAMP(1);                                   // repr stages
    // reload the representation's sets; in flight under step 1's first RO stages
    sm_load<SM_MAX_SIM>(RO, RO + P.n_root < P.n_sim ? RO + P.n_root : P.n_sim, io.w_sim, wr, P.nzm, P.zero16);
    SM_STAMP(2);                                   // sim reload (issue only)
    for (int i = 1; i <= K; ++i) {
        // make_dynamics_input (:293-304) fused into the first stage: it reads
        // h_{i-1} (h_out, written by the previous step's last stage, a barrier
        // ago) and the step's a/|A|
        const SmFusedIn fin{act + P.h_out, nullptr, nullptr, aval + (i - 1), K + 1, H, P.plane, P.x_pred, P.x_dyn};
        SM_STAMP(3);                               // step inputs (none left: fused)
        sm_run<T, SM_MAX_SIM, 2, 0, BNM>(P.n_sim, wr, rec_sim, act, &fin, bn_sim);
        SM_STAMP(4);                               // the 8 stages
        // raw outputs (logits, value, reward before their read-out
        // activations); mz_learner_grad_kernel applies softmax / tanh for all
        // (sample, step) pairs in parallel
        if (tid < T * (A + 2) && tile0 + o_gl < P.B) {
            const int gl = o_gl, c = o_c;
            const int bb = tile0 + gl;
            float x;
            float* dst;
            float* dst0 = nullptr;
            if (c < A) {
                x = act[P.p_out + c * T + gl];
                dst = io.pp + ((size_t)bb * (K + 1) + i) * A + c;
                if (i == 1) dst0 = io.pp + ((size_t)bb * (K + 1)) * A + c;
            } else if (c == A) {
                x = act[P.v_out + gl];
                dst = io.pv + (size_t)bb * (K + 1) + i;
                if (i == 1) dst0 = io.pv + (size_t)bb * (K + 1);
            } else {
                x = act[P.r_out + gl];
                dst = io.pr + (size_t)bb * (K + 1) + i;
                if (i == 1) io.pr[(size_t)bb * (K + 1)] = 0.0f;   // raw 0: every read-out maps 0 to 0
            }
            *dst = x;
            if (dst0) *dst0 = x;
        }
        // the next step's input copy reads h_out and writes x_pred / x_dyn,
        // which nothing above reads: no barrier needed here
        SM_STAMP(5);                               // raw output writes
    }
#ifdef MZ_STAMPS
    if (threadIdx.x == 0 && P.stamps)
        for (int i = 0; i < 8; ++i) P.stamps[lb * 8 + i] = st_acc[i];
#endif
}

extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_unroll_small1(SmallUnrollParams P) { unroll_body<1, 0>(P, blockIdx.x, sm_io(P)); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_unroll_small2(SmallUnrollParams P) { unroll_body<2, 0>(P, blockIdx.x, sm_io(P)); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_unroll_small1_bn(SmallUnrollParams P) { unroll_body<1, 1>(P, blockIdx.x, sm_io(P)); }
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_unroll_small2_bn(SmallUnrollParams P) { unroll_body<2, 1>(P, blockIdx.x, sm_io(P)); }

// One learner iteration in one launch (LearnParams): unroll (+ get_batch) and
// each tile's loss terms ‖ Σθ² + ADAM into the second image set; last block
// folds.  Same results as mz_unroll_small* + mz_learner_grad_kernel (fused
// ADAM): the loss terms, the θ² slices (256-thread groups) and the fold are
// the same code on the same decomposition.
template <int T, int BNM>
__device__ __forceinline__ void learn_body(const SmallUnrollParams& P, const LearnParams& L) {
    __shared__ float stg[SM_THREADS];
    __shared__ double red[SM_THREADS];
    const int tid = threadIdx.x;
    const int K1 = P.K + 1, n = P.B * K1;
    float* vsq = L.terms;
    float* cet = L.terms + n;
#ifdef MZ_STAMPS
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
    // logical block: with L.xcd the unroll workgroups are the physical blocks
    // 0, 8, 16, .. (one XCD under round-robin dispatch: their weight image is
    // fetched into one L2), the other roles take the remaining blocks in order
    const int pb = (int)blockIdx.x;
    const int lb = L.xcd ? ((pb & 7) == 0 ? pb >> 3 : L.nU + pb - (pb >> 3) - 1) : pb;
    if (lb < L.nU) {
        unroll_body<T, BNM>(P, lb, sm_io(P));
#ifdef MZ_STAMPS
        const unsigned long long t_unroll = __builtin_amdgcn_s_memtime();
#endif
        __syncthreads();                               // the tile's raw outputs -> its loss groups
        const int g16 = tid >> 4, a = tid & 15, gl = g16 / K1, k = g16 - gl * K1;
        const int b = lb * T + gl;
        if (gl < T && b < P.B)
            lg_step_terms<16>(b * K1 + k, a, P.A, P.v_act, P.r_act, P.pv, P.pp, P.pr, L.tv, L.tp, vsq, cet,
                              stg + (tid & ~15));
#ifdef MZ_STAMPS   // slot 6: unroll start -> end, slot 7: loss terms (wave 0)
        if (tid == 0 && P.stamps) {
            P.stamps[lb * 8 + 6] = t_unroll - t_start;
            P.stamps[lb * 8 + 7] = __builtin_amdgcn_s_memtime() - t_unroll;
        }
#endif
    } else if (lb >= L.nU + LEARN_L2_GROUPS) {
        // the next step's get_batch into the other batch set (read by the next launch;
        // blocks past the last sample are idle)
        const int b = (lb - L.nU - LEARN_L2_GROUPS) * (SM_THREADS / 64) + (tid >> 6);
        if (b < L.pfq.B && L.pf_nb > 0) rp_sample_one(L.pfq, b, tid & 63);
        if (lb == L.nU + LEARN_L2_GROUPS && L.pf_nb > 0 && tid == 0) {
            L.pf_hdr_next[0] = L.pf_epoch;
            L.pf_hdr_next[1] = L.pfq.counters[0];
            L.pf_hdr_next[2] = (long long)L.pfq.step;
            L.pf_hdr_next[3] = (long long)L.pfq.B;
        }
    } else {
        const int half = tid >> 8, t256 = tid & (MZ_THREADS - 1);
        for (int pass = 0; pass < LEARN_L2_PASSES; ++pass) {       // (block-uniform trip count: barriers inside)
            const int vb = (pass * LEARN_L2_GROUPS + lb - L.nU) * SM_SLOTS + half;
            const bool vin = vb < 3 * MZ_L2_BLOCKS;
            const int net = vb / MZ_L2_BLOCKS, blk = vb % MZ_L2_BLOCKS;
            red[tid] = vin ? lg_l2_slice(net, blk, t256, L.netoff, L.flat, nullptr, L.ad) : 0.0;
            __syncthreads();
            for (int o = MZ_THREADS / 2; o > 0; o >>= 1) {        // lg_tree256 on each half
                if (t256 < o) red[tid] += red[tid + o];
                __syncthreads();
            }
            if (t256 == 0 && vin)                  // agent scope: read by the fold (lg_fold)
                __hip_atomic_store(L.part + net * MZ_L2_BLOCKS + blk, red[tid], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();                       // red[] reused by the next pass
        }
    }
    lg_fold(P.B, P.K, vsq, cet, L.gscale, nullptr, L.part, L.counter, L.out);
}

extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_small1(SmallUnrollParams P, LearnParams L) {
    learn_body<1, 0>(P, L);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_small2(SmallUnrollParams P, LearnParams L) {
    learn_body<2, 0>(P, L);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_small1_bn(SmallUnrollParams P, LearnParams L) {
    learn_body<1, 1>(P, L);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_small2_bn(SmallUnrollParams P, LearnParams L) {
    learn_body<2, 1>(P, L);
}


// ------------------------------------------------ L learner steps per launch pair
// (ChainParams / LearnMultiParams, mz_small_params.h)
// one parameter p's L ADAM iterations in registers; its θ_{t+i} feed step t+i's Σθ² (added to
// rd[i·MZ_THREADS] in place, or with HELP stored to hx[i·hx_n] for the slot's last block); CAP: θ after steps
// cap_i[0] / cap_i[1] also copied out (a separate instance: the plain chain carries no per-step tests)
template <bool CAP, bool HELP>
__device__ __forceinline__ void chain_param(const ChainParams& C, size_t p, double* rd, float* hx,
                                            const double (*sbp)[MZ_MULTI_MAX]) {
    const int L = C.L;
    float x = C.flat[p], m = C.M[p], v = C.V[p];
    const int it = C.inv_tile[p], is = C.inv_small[p];
    const bool sbank = C.bank_w != nullptr, tbank = C.tbank_w != nullptr;   // (uniform)
    for (int i = 0; i < L; ++i) {
        if constexpr (HELP) __hip_atomic_store(hx + (size_t)i * C.hx_n, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else rd[i * MZ_THREADS] += (double)x * (double)x;           // step t+i's Σθ² reads θ_{t+i}
#ifndef MZ_DBG_NO_BANK   // diagnostic only (wrong results): the chain without the bank scatter
        if (sbank) mz_scatter(x, is, C.bank_w + i * C.bws, C.bank_b + i * C.bbs);
#endif
        if (tbank) mz_scatter(x, it, C.tbank_w + i * C.tws, C.tbank_b + i * C.tbs);
        if (C.fbank) C.fbank[i * C.fstride + p] = x;
#ifdef MZ_DBG_CHEAP_ADAM   // diagnostic only (wrong results): the chain without ADAM's f64 arithmetic
        x = x * 0.999f + (float)sbp[2][i];
#else
        x = adam_2theta(x, m, v, sbp[0][i], sbp[1][i], sbp[2][i]);   // Learning.jl:395-397
#endif
        if (C.theta) C.theta[i * C.nflat + p] = x;
        if constexpr (CAP) {
            if (i == C.cap_i[0]) {
                C.cap_dst[0][p] = x;
                if (C.cap_img[0]) {                         // (the actors' images: no repack after the call)
                    mz_scatter(x, it, C.cap_img[0], C.cap_img[1]);
                    mz_scatter(x, is, C.cap_img[2], C.cap_img[3]);
                }
            }
            if (i == C.cap_i[1]) C.cap_dst[1][p] = x;
        }
    }
    C.flat[p] = x; C.M[p] = m; C.V[p] = v;
    mz_scatter(x, it, C.Wp, C.Bp);
    mz_scatter(x, is, C.smw, C.smb);
}

// this thread's parameters of slice (net, sb): e = sb·256 + tid + k·stride in k order
template <bool CAP>
__device__ __forceinline__ void chain_slice(const ChainParams& C, int net, int sb, double (*red)[MZ_THREADS],
                                            double (*sbp)[MZ_MULTI_MAX]) {
    const int tid = threadIdx.x;
    const size_t off = C.netoff[net], cnt = C.netoff[3 + net];
    const size_t stride = (size_t)MZ_L2_BLOCKS * MZ_THREADS;
    for (size_t e = (size_t)sb * MZ_THREADS + tid; e < cnt; e += stride) {
        chain_param<CAP, false>(C, off + e, &red[0][tid], nullptr, sbp);
#ifdef MZ_DBG_ONE_ELEM   // diagnostic only (wrong results): each thread's first parameter alone
        break;
#endif
    }
}

// lg_tree256 per step: level o adds red[i][j + o] into red[i][j] for j < o, every step i; the o·L adds of
// a level are spread over all 256 threads (each the same add as the per-step tree's, so the same bits),
// not L in sequence on the first o threads; step i's sum -> part[i·NSL]
__device__ __forceinline__ void chain_tree(double (*red)[MZ_THREADS], int L, double* part) {
    const int tid = threadIdx.x;
    for (int o = MZ_THREADS / 2; o > 0; o >>= 1) {
        for (int x = tid; x < o * L; x += MZ_THREADS) {
            const int i = x / o, j = x - i * o;
            red[i][j] += red[i][j + o];
        }
        __syncthreads();
    }
    if (tid < L) part[(size_t)tid * 3 * MZ_L2_BLOCKS] = red[tid][0];
}

// slot (net, sb)'s blocks: the slice and its helpers (k − 1)·128 + sb, k >= 1
__device__ __forceinline__ int chain_npart(const ChainParams& C, int net, int sb) {
    return 1 + (C.nh[net] > sb ? (C.nh[net] - 1 - sb) / MZ_L2_BLOCKS + 1 : 0);
}

// a block of a slot with helpers: its θ stores performed, it counts itself in (agent scope); the last of
// the slot's blocks (the counter reaches a multiple of npart) forms the slot's per-step Σθ²
// from every parameter's stored θ_{t+i}, in lg_l2_slice's k order, and its tree.  No block waits for
// another, so the launch completes whatever else shares the GPU.
__device__ __forceinline__ void chain_arrive(const ChainParams& C, int net, int sb, double (*red)[MZ_THREADS],
                                             int* last) {
    const int tid = threadIdx.x, L = C.L;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                // this wave's θ stores performed
    __syncthreads();
    if (tid == 0) {
        const unsigned long long np = (unsigned long long)chain_npart(C, net, sb);
        const unsigned long long old = __hip_atomic_fetch_add(C.hcnt + net * MZ_L2_BLOCKS + sb, 1ull,
                                                              __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        *last = (old + 1) % np == 0;                  // (np arrivals per launch: self-aligning)
    }
    __syncthreads();
    if (!*last) return;
    const size_t cnt = C.netoff[3 + net], stride = (size_t)MZ_L2_BLOCKS * MZ_THREADS;
    // (the MZ_MULTI_MAX rows of hx are all allocated: the loads are issued together, sc1 like the stores)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(C.hx, (short)0, (int)(MZ_MULTI_MAX * C.hx_n * 4), 0x00020000);
    for (int i = 0; i < L; ++i) red[i][tid] = 0.0;
    for (size_t e = (size_t)sb * MZ_THREADS + tid; e < cnt; e += stride) {
        const int b0 = (int)((C.hoff[net] + e) * 4);
        float xv[MZ_MULTI_MAX];
#pragma unroll
        for (int i = 0; i < MZ_MULTI_MAX; ++i)
            xv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, b0 + (int)(i * C.hx_n * 4), 0, 16));
#pragma unroll
        for (int i = 0; i < MZ_MULTI_MAX; ++i)
            if (i < L) red[i][tid] += (double)xv[i] * (double)xv[i];
    }
    __syncthreads();
    chain_tree(red, L, C.part + net * MZ_L2_BLOCKS + sb);
}

// mz_learn_chain: blocks [0, nh) are the helpers (ChainParams::nh), then
// [nh, nh + 3·MZ_L2_BLOCKS) lg_l2_slice's slices (net, blk): each thread runs its
// parameters' L ADAM iterations (∇ = 2θ, Q11) in registers and keeps one
// Σθ_{t+i}² per step in lg_l2_slice's order; the per-step trees are
// lg_tree256's, level by level.  The blocks after them draw the L batches.
// The chain and the unroll launches run one after another in stream order
// (a two-stream variant that overlapped them measured slower, mz_engine.hip
// learner_multi).
extern "C" __global__ __launch_bounds__(MZ_THREADS) void mz_learn_chain(ChainParams C) {
    // per step i: this thread's Σθ_{t+i}² (accumulated in place in LDS: no
    // register array indexed by the runtime step)
    __shared__ double red[MZ_MULTI_MAX][MZ_THREADS];
    __shared__ double sbp[3][MZ_MULTI_MAX];         // β1^t, β2^t, η of step t+i
    __shared__ int last;
    const int tid = threadIdx.x, nht = C.nh[0] + C.nh[1] + C.nh[2];
    const int blk = (int)blockIdx.x - nht;
    constexpr int NSL = 3 * MZ_L2_BLOCKS;
    const size_t stride = (size_t)MZ_L2_BLOCKS * MZ_THREADS;
    const int L = C.L;
    const bool cap = C.cap_i[0] >= 0 || C.cap_i[1] >= 0;   // (mz_train_run's refresh steps in this chain)
    if (blk >= NSL) {                               // get_batch of step t+i, sample b (ReplayBuffer.jl:188-217)
        const int q = (blk - NSL) * (MZ_THREADS / 64) + (tid >> 6);
        if (q >= L * C.B) return;
        const int i = q / C.B, b = q - i * C.B;
        RpSampleParams Q = C.q;
        Q.step += (uint32_t)i;
        Q.obs += i * C.s_obs; Q.actions += i * C.s_k1; Q.tv += i * C.s_k1; Q.tr += i * C.s_k1;
        Q.tpol += i * C.s_tp; Q.gscale += (size_t)i * C.B; Q.index += (size_t)i * 2 * C.B;
        rp_sample_one(Q, b, tid & 63);
        return;
    }
    if (tid < MZ_MULTI_MAX) { sbp[0][tid] = C.bp1[tid]; sbp[1][tid] = C.bp2[tid]; sbp[2][tid] = C.eta[tid]; }
    __syncthreads();
    // a helper (blk < 0: helper hb of net n, parameter e = stride + hb·256 + tid) or the slice of a slot
    // with helpers: θ stored, the slot's last block sums
    int net, sb;
    size_t e;
    if (blk < 0) {
        int hb = (int)blockIdx.x;
        net = 0;
        while (hb >= C.nh[net]) hb -= C.nh[net++];
        e = stride + (size_t)hb * MZ_THREADS + tid;
        sb = hb % MZ_L2_BLOCKS;
    } else {
        net = blk / MZ_L2_BLOCKS;
        sb = blk - net * MZ_L2_BLOCKS;
        e = (size_t)sb * MZ_THREADS + tid;
    }
    if (blk < 0 || chain_npart(C, net, sb) > 1) {
        if (e < C.netoff[3 + net]) {
            float* hx = C.hx + C.hoff[net] + e;
            if (cap) chain_param<true, true>(C, C.netoff[net] + e, nullptr, hx, sbp);
            else chain_param<false, true>(C, C.netoff[net] + e, nullptr, hx, sbp);
        }
        chain_arrive(C, net, sb, red, &last);
        return;
    }
    for (int i = 0; i < L; ++i) red[i][tid] = 0.0;
    __syncthreads();
    if (cap) chain_slice<true>(C, net, sb, red, sbp);
    else chain_slice<false>(C, net, sb, red, sbp);
    __syncthreads();
    chain_tree(red, L, C.part + blk);
}

// mz_learn_multi{1,2}: workgroup (step i, tile lb).  With M.xcd, step i's
// workgroups are the physical blocks on XCD i mod 8 (round-robin dispatch), so
// each XCD's L2 holds its steps' bank images only.
template <int T, int BNM>
__device__ __forceinline__ void learn_multi_body(const SmallUnrollParams& P, const LearnMultiParams& M) {
    __shared__ float stg[SM_THREADS];
    const int tid = threadIdx.x, pb = (int)blockIdx.x;
    int i, lb;
    if (M.xcd) {
        const int r = pb >> 3;
        i = (pb & 7) + 8 * (r / M.nU);
        lb = r % M.nU;
    } else {
        i = pb / M.nU;
        lb = pb - i * M.nU;
    }
    if (i >= M.L) return;                           // (xcd grids round L up to a multiple of 8)
    const int K1 = P.K + 1;
    if (M.sample) {                                 // get_batch of step t+i (ReplayBuffer.jl:188-217), this tile
        const int w = tid >> 6, b = lb * T + w;
        if (w < T && b < P.B) {
            RpSampleParams Q = M.q;
            Q.step += (uint32_t)i;
            Q.obs += i * M.s_obs; Q.actions += i * M.s_k1; Q.tv += i * M.s_k1; Q.tr += i * M.s_k1;
            Q.tpol += i * M.s_tp; Q.gscale += (size_t)i * P.B; Q.index += (size_t)i * 2 * P.B;
            rp_sample_one(Q, b, tid & 63);
        }
        __threadfence_block();
        __syncthreads();
    }
    SmIO io;
    io.obs = M.obs + i * M.s_obs; io.actions = M.act + i * M.s_k1;
    io.pv = M.pv + i * M.s_k1; io.pp = M.pp + i * M.s_tp; io.pr = M.pr + i * M.s_k1;
    io.w_sim = M.bank_w + i * M.bws;
    io.w_root = io.w_sim + (size_t)P.n_sim * SM_SLOTS * 256 * 16;
    io.bias = M.bank_b + i * M.bbs;
    unroll_body<T, BNM>(P, lb, io);
    __syncthreads();                                // the tile's raw outputs -> its loss groups
    float* vsq = M.terms + 2 * i * M.s_k1;
    float* cet = vsq + M.s_k1;
    const int g16 = tid >> 4, a = tid & 15, gl = g16 / K1, k = g16 - gl * K1;
    const int b = lb * T + gl;
    if (gl < T && b < P.B)
        lg_step_terms<16>(b * K1 + k, a, P.A, P.v_act, P.r_act, io.pv, io.pp, io.pr, M.tv + i * M.s_k1,
                          M.tp + i * M.s_tp, vsq, cet, stg + (tid & ~15));
    lg_fold(P.B, P.K, vsq, cet, M.gs + (size_t)i * P.B, nullptr, M.part + (size_t)i * 3 * MZ_L2_BLOCKS,
            M.counter + i * MZ_MULTI_CNT_STRIDE, M.out_last && i == M.L - 1 ? M.out_last : M.out + 8 * i,
            (unsigned)M.nU);
}

extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi1(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<1, 0>(P, M);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi2(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<2, 0>(P, M);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi4(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<4, 0>(P, M);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi4_bn(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<4, 1>(P, M);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi1_bn(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<1, 1>(P, M);
}
extern "C" __global__ __launch_bounds__(SM_THREADS, 1) void mz_learn_multi2_bn(SmallUnrollParams P, LearnMultiParams M) {
    learn_multi_body<2, 1>(P, M);
}
