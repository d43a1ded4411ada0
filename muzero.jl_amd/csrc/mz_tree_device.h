// mz_tree_device.h — the MCTS tree phases shared by the search kernels
// (SelfPlay.jl:88-217, 293-306): select, expand, backup, search statistics.
//
// Tree of one game (slot e = 0 is the root, e = s+1 the node expanded by
// simulation s; edge (e, a) = child a of expanded node e).  Edge i = e*A + a
// is one 16-byte record (a single ds_read_b128 in select):
//   .nc  u32  visit count N (low 16 bits) | child slot + 1 (high 16; 0 = none)
//   .w   f32  value_sum of the child
//   .p   f32  prior of the child
//   .ev  f32  the child's value term of ucb_score (SelfPlay.jl:176-181),
//             R_c + γ·(±W/N), written by backup with the exact f32 ops select
//             would evaluate (valid when N > 0)
// and per expanded node
//   nr[e]  f32  reward of expanded node e (node.reward)
//   ntp[e] i8   to_play of expanded node e
// The same code runs on an LDS or an HBM copy.
// Threads are grouped GW lanes per game (lane a = child slot a, A <= GW):
// GW = 16 (one DPP row; every FC kernel and A <= 16) or 32 (two rows, A <= 32,
// e.g. the 18 Atari actions of BASELINE configs[4]).
#pragma once
#include "mz_internal.h"

struct TreeView {
    float4* e;          // edge records {nc bits, w, p, ev}
    float* nr;
    int8_t* ntp;
    __device__ __forceinline__ uint32_t& nc(int i) const { return reinterpret_cast<uint32_t*>(e + i)[0]; }
    __device__ __forceinline__ float& w(int i) const { return reinterpret_cast<float*>(e + i)[1]; }
    __device__ __forceinline__ float& p(int i) const { return reinterpret_cast<float*>(e + i)[2]; }
    __device__ __forceinline__ float& ev(int i) const { return reinterpret_cast<float*>(e + i)[3]; }
};

__host__ __device__ __forceinline__ size_t tree_bytes(int E, int NN) {
    return (16 * (size_t)E + 4 * (size_t)NN + (size_t)NN + 15) & ~(size_t)15;
}

__device__ __forceinline__ TreeView tree_view(char* base, int E, int NN) {
    TreeView t;
    t.e = reinterpret_cast<float4*>(base);
    t.nr = reinterpret_cast<float*>(base + 16 * (size_t)E);
    t.ntp = reinterpret_cast<int8_t*>(base + 16 * (size_t)E + 4 * (size_t)NN);
    return t;
}

// max over the 16-lane group (= one DPP row): quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror.  Exact (comparisons only).
__device__ __forceinline__ float dpp_f(float v, int ctrl) {
    switch (ctrl) {
        case 0xB1: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
        case 0x4E: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
        case 0x141: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
        default: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
    }
}
__device__ __forceinline__ float g16_max(float v) {
    float t;
    t = dpp_f(v, 0xB1); v = v > t ? v : t;
    t = dpp_f(v, 0x4E); v = v > t ? v : t;
    t = dpp_f(v, 0x141); v = v > t ? v : t;
    t = dpp_f(v, 0x140); v = v > t ? v : t;
    return v;
}
__device__ __forceinline__ float g16_min(float v) {
    float t;
    t = dpp_f(v, 0xB1); v = v < t ? v : t;
    t = dpp_f(v, 0x4E); v = v < t ? v : t;
    t = dpp_f(v, 0x141); v = v < t ? v : t;
    t = dpp_f(v, 0x140); v = v < t ? v : t;
    return v;
}

// OR over the 16-lane group (same DPP pattern): used to broadcast the value
// held by exactly one lane (the others contribute 0).
__device__ __forceinline__ uint32_t g16_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return v;
}

__device__ __forceinline__ int g16_isum(int v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}

// GW-lane group versions: the 16-lane DPP reduction, then for GW = 32 one
// exchange with the other row of the pair.  The row pair of a GW = 32 group (rows 0/1 or 2/3) exchanges through
// v_permlane16_swap (gfx950, VALU): with both operands equal the two results
// are {own row, partner row} in row order, in every lane of the pair.
__device__ __forceinline__ void row_pair(uint32_t v, uint32_t& x, uint32_t& y) {
    const auto s = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    x = (uint32_t)s[0]; y = (uint32_t)s[1];
}
template <int GW> __device__ __forceinline__ float gmax(float v) {
    v = g16_max(v);
    if constexpr (GW == 32) {
        uint32_t x, y;
        row_pair(__builtin_bit_cast(uint32_t, v), x, y);
        const float fx = __builtin_bit_cast(float, x), fy = __builtin_bit_cast(float, y);
        v = fx > fy ? fx : fy;
    }
    return v;
}
template <int GW> __device__ __forceinline__ float gmin(float v) {
    v = g16_min(v);
    if constexpr (GW == 32) {
        uint32_t x, y;
        row_pair(__builtin_bit_cast(uint32_t, v), x, y);
        const float fx = __builtin_bit_cast(float, x), fy = __builtin_bit_cast(float, y);
        v = fx < fy ? fx : fy;
    }
    return v;
}
template <int GW> __device__ __forceinline__ uint32_t gor(uint32_t v) {
    v = g16_or(v);
    if constexpr (GW == 32) { uint32_t x, y; row_pair(v, x, y); v = x | y; }
    return v;
}
template <int GW> __device__ __forceinline__ int gisum(int v) {
#pragma unroll
    for (int o = GW / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, GW);
    return v;
}

// sequential (ascending) f32 sum of lanes 0..n-1 of the GW-lane group; every
// lane returns the same value (the oracle's `s = s + y[i]` loop order).  The
// values are staged through this group's GW-float LDS slot `st` (same wave:
// LDS ops complete in order) and read back as GW/4 broadcast b128 loads.
// Every caller's lanes n..GW-1 hold +0, and a partial sum that starts at +0 is
// never -0 (x + -0 = x for x = +0 in round-to-nearest), so adding them is exact:
// the sum runs in blocks of four, a block skipped by a wave-uniform branch once
// it starts past n — a plain dependent add chain, with no per-element select.
template <int GW>
__device__ __forceinline__ float gseqsum(float v, int n, float* st, int a) {
    st[a] = v;
    __builtin_amdgcn_wave_barrier();
    float x[GW];
#pragma unroll
    for (int b = 0; b < GW; b += 4) {
        const float4 q = *reinterpret_cast<const float4*>(st + b);
        x[b] = q.x; x[b + 1] = q.y; x[b + 2] = q.z; x[b + 3] = q.w;
    }
    __builtin_amdgcn_wave_barrier();
    const int nu = __builtin_amdgcn_readfirstlane(n);
    float s = x[0] + 0.0f;                  // (= 0.0f + x[0], the oracle's first step)
    s = s + x[1]; s = s + x[2]; s = s + x[3];
#pragma unroll
    for (int b = 4; b < GW; b += 4)
        if (b < nu) { s = s + x[b]; s = s + x[b + 1]; s = s + x[b + 2]; s = s + x[b + 3]; }
    return s;
}
__device__ __forceinline__ float g16_seqsum(float v, int n, float* st, int a) { return gseqsum<16>(v, n, st, a); }

__device__ __forceinline__ int nth_set_bit(uint32_t m, int k) {
    for (int i = 0; i < k; ++i) m &= m - 1;
    return __builtin_ctz(m);
}

// expand_node! (SelfPlay.jl:88-96) priors for the GW-lane group: the policy
// head's softmax over all A logits (Learning.jl:114), then the softmax over
// the legal entries (:89, Q3).  `logit` is this lane's logit (a < A).
template <int GW = 16>
__device__ __forceinline__ float double_softmax_prior(float logit, int a, int A, uint32_t legal, float* st) {
    const bool in = a < A;
    const float x = in ? logit : -INFINITY;
    const float m = gmax<GW>(x);
    const float ex = in ? det_expf(x - m) : 0.0f;
    const float s = gseqsum<GW>(ex, A, st, a);
    const float prob = in ? ex / s : 0.0f;
    const bool lg = in && ((legal >> a) & 1u);
    const float m2 = gmax<GW>(lg ? prob : -INFINITY);
    const float e2 = lg ? det_expf(prob - m2) : 0.0f;
    const float s2 = gseqsum<GW>(e2, A, st, a);  // illegal lanes add +0: same as the legal-only sum
    return lg ? e2 / s2 : 0.0f;
}

// add_exploration_noise! (SelfPlay.jl:102-109) noise for the GW-lane group,
// lane-parallel: legal lane a draws Dirichlet component rank(a) from its own
// stream (mz_dirichlet_gamma); the f32 sum runs in ascending action order
// (illegal lanes add +0, exact); returns the normalised noise (0 if illegal).
template <int GW = 16>
__device__ __forceinline__ float root_noise_lane(uint32_t legal, int a, int A, uint64_t seed, uint32_t gid,
                                                 uint32_t step, float alpha, float* st) {
    const bool lg = a < A && ((legal >> a) & 1u);
    const int r = __builtin_popcount(legal & ((1u << a) - 1u));
    const float gm = lg ? mz_dirichlet_gamma(seed, gid, step, r, alpha) : 0.0f;
    const float sum = gseqsum<GW>(gm, A, st, a);
    const float inv = 1.0f / sum;
    return lg ? gm * inv : 0.0f;
}

// Write the A child edges of expanded slot e (N=0, W=0, prior, no child).
__device__ __forceinline__ void init_edges(const TreeView& t, int e, int a, int A, float prior) {
    if (a < A) {
        const int i = e * A + a;
        t.e[i] = make_float4(0.0f, 0.0f, prior, 0.0f);     // nc = 0 (bits), w = 0, p, ev
    }
}

struct SelectOut { int leaf_e, leaf_a, vtp, depth; };

// Path of one simulation: path[2d] = edge index e*A + a taken at depth d,
// path[2d+1] = child slot it leads to (-1 for the leaf until expanded).

// pb_term table index: the host tabulates pbc(Np) * (sqrt(Np) / (Nc + 1))
// (the f64 subexpression of ucb_score, SelfPlay.jl:172-174) for Nc < Np <=
// S+1 as a triangle, so select replaces an f64 division by one LDS read.
__host__ __device__ __forceinline__ int pbterm_index(int Np, int Nc) {
#ifdef __HIP_DEVICE_COMPILE__
    return (int)(__umul24((unsigned)Np, (unsigned)(Np + 1)) >> 1) + Nc;   // full-rate 24-bit multiply
#else
    return (int)(((unsigned)Np * (unsigned)(Np + 1)) >> 1) + Nc;
#endif
}
__host__ __device__ __forceinline__ size_t pbterm_count(int S) { return (size_t)(S + 2) * (S + 3) / 2; }

// max over the 16-lane group, one v_max_f32_dpp per step (the hazard pad —
// a DPP read of a VGPR written by the previous VALU needs 2 wait states — is
// inside the string).  For select's argmax this equals g16_max: no NaNs
// occur, and -0/+0 compare equal in the tie test that follows.
__device__ __forceinline__ float g16_vmax(float v) {
    asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1"
                 : "+v"(v));
    return v;
}

// g16_vmax into a fresh register (the first step reads u through DPP, so no
// copy of u is made); no pad after the last step, whose consumer (the tie
// compare) is not a DPP instruction.
__device__ __forceinline__ float g16_vmax_to(float u) {
    float m;
    asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
                 : "=&v"(m) : "v"(u));
    return m;
}

// select_child loop (SelfPlay.jl:256-268) for the game of this GW-lane group.
// pUCT (ucb_score :171-184) in f64 with one rounding to f32 (Q5); ties by
// exact equality, broken by the Philox TIE stream keyed (sim, depth) — the
// draw only matters (and is only computed) when there is more than one tie.
// Per level: one LDS round trip (the 16-byte edge record, then the pb_term
// entry when TAB, else the pbc/sqrt entries and an f64 division), a
// branch-free score (illegal lanes score a clamped real edge and are masked
// to -inf), a DPP max, a ballot, and the chosen edge's record by DPP.  The
// path stays in registers while depth < GW (lane d keeps level d) and is
// written to `path` once at the end; deeper levels are stored directly.
// NGRP: GW-lane groups in use in this wave (GW = 16: the argmax lane and the
// chosen record are then found per group with scalar ops on the ballot and a
// readlane, instead of per-lane shifts and a DPP OR chain).
template <bool TAB, int GW = 16, int NGRP = 4>
__device__ __forceinline__ SelectOut select_path(const TreeView& t, int* path, int root_N, int root_tp,
                                                 uint32_t legal, float mmin, float mmax, int a, int lane,
                                                 int A, int players, float discount, const double* pbterm,
                                                 const double* pbc_tab, const double* sqrt_tab, uint64_t seed,
                                                 uint32_t gid, uint32_t step, int sim) {
    const bool lg = a < A && ((legal >> a) & 1u);
    const bool norm = mmax > mmin;
    const float den = mmax - mmin;
    const int ac = a < A ? a : A - 1;
    int e = 0, Np = root_N, depth = 0, vtp = root_tp;
    int pe = 0, pc = 0;
    const uint64_t lgmask = __builtin_amdgcn_ballot_w64(lg);
    SelectOut out;
    for (;;) {
        // the parent's pUCT table entries depend only on Np: read them with the record
        double pbn = 0.0, sqn = 0.0;
        if constexpr (!TAB) { pbn = pbc_tab[Np]; sqn = sqrt_tab[Np]; }
        // the pb_term row of the parent depends on Np alone: formed while the
        // record is in flight
        const double* prow = TAB ? pbterm + (__umul24((unsigned)Np, (unsigned)(Np + 1)) >> 1) : nullptr;
        float4 ed = t.e[(int)__umul24((unsigned)e, (unsigned)A) + ac];
        // keep the whole record one load and the score branch-free: without
        // these the compiler sinks the ev load and the division into an
        // Nc > 0 branch (a second LDS round trip and two exec branches)
        asm volatile("" : "+v"(ed.x), "+v"(ed.y), "+v"(ed.z), "+v"(ed.w));
        if constexpr (!TAB) asm volatile("" : "+v"(pbn), "+v"(sqn));
        const uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
        const int Nc = (int)(nc & 0xffffu);
        double pb_c;
        float num = ed.w - mmin;
        if constexpr (TAB) {
            pb_c = prow[Nc < Np ? Nc : Np];               // pbterm[pbterm_index(Np, min(Nc, Np))]
            // the read is issued here (memory clobber) and the division below
            // depends on this asm: it runs while the entry is in flight
            asm volatile("" : "+v"(num) :: "memory");
        } else {
            pb_c = pbn * (sqn / (double)(Nc + 1));
        }
        // normalize (:33-39), the IEEE division: a reciprocal per walk plus a
        // Markstein correction is exact on [2^-60, 2^60] but needs a per-level
        // range test and branch, which measured slower
        float vn = num / den;                            // discarded unless norm and Nc > 0
        asm volatile("" : "+v"(vn));                     // (unconditional: not sunk into an Nc > 0 branch)
        const float vs = Nc > 0 ? (norm ? vn : ed.w) : 0.0f;
        double pz = (double)ed.z, vsd = (double)vs;      // ready before the pb_term entry lands
        asm volatile("" : "+v"(pz), "+v"(vsd), "+v"(pb_c));
        const double prior_score = pb_c * pz;
        const float us = (float)(prior_score + vsd);
        const float u = lg ? us : -INFINITY;
        // GW = 32: the padded form (its consumer is the row-pair permlane)
        float m = GW == 16 ? g16_vmax_to(u) : g16_vmax(u);
        if constexpr (GW == 32) {
            uint32_t x, y;
            row_pair(__builtin_bit_cast(uint32_t, m), x, y);
            const float fx = __builtin_bit_cast(float, x), fy = __builtin_bit_cast(float, y);
            m = fx > fy ? fx : fy;
        }
        // ballot(lg && u == m): one compare into an SGPR pair and a scalar AND
        // with the walk-invariant legal mask (the builtin form compiled to a
        // compare, a select and a second compare on the per-level chain)
        uint64_t eqm;
        asm volatile("v_cmp_eq_f32_e64 %0, %1, %2" : "=s"(eqm) : "v"(u), "v"(m));
        const uint64_t bal = eqm & lgmask;
        depth += 1;
        int ach;
        uint32_t ncc;
        if constexpr (GW == 16) {
            // per group g: its candidate mask, first candidate and whether it ties
            // (wave-uniform, scalar); each lane takes its group's by select
            const int grp = lane >> 4;
            uint32_t gm[NGRP];
            int gf[NGRP];
            bool tie = false;
#pragma unroll
            for (int g = 0; g < NGRP; ++g) {
                gm[g] = (uint32_t)(bal >> (16 * g)) & 0xffffu;
                gf[g] = __builtin_ctz(gm[g] | 0x10000u);
                tie |= (gm[g] & (gm[g] - 1)) != 0;
            }
            ach = gf[0];
#pragma unroll
            for (int g = 1; g < NGRP; ++g) ach = grp == g ? gf[g] : ach;
            if (tie) {                                    // ties (rare): the Philox draw per group
                uint32_t mask = gm[0];
#pragma unroll
                for (int g = 1; g < NGRP; ++g) mask = grp == g ? gm[g] : mask;
                const int nt = __builtin_popcount(mask);
                if (nt > 1) {
                    const uint32_t r = mz_rng_u32(seed, MZ_RNG_TIE, gid, step, ((uint32_t)sim << 12) | (uint32_t)depth);
                    ach = nth_set_bit(mask, (int)mz_rng_below(r, (uint32_t)nt));
                }
                ncc = g16_or(a == ach ? nc : 0u);
            } else {                                      // the chosen lane's nc by readlane
                ncc = (uint32_t)__builtin_amdgcn_readlane((int)nc, gf[0]);
#pragma unroll
                for (int g = 1; g < NGRP; ++g) {
                    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)nc, 16 * g + (gf[g] & 15));
                    ncc = grp == g ? v : ncc;
                }
            }
        } else {
            const uint32_t mask = (uint32_t)(bal >> (lane & 32));
            ach = __builtin_ctz(mask);
            // ties (rare): one wave-uniform test, then the Philox draw per group
            if (__builtin_amdgcn_ballot_w64((mask & (mask - 1)) != 0) != 0) {
                const int nt = __builtin_popcount(mask);
                if (nt > 1) {
                    const uint32_t r = mz_rng_u32(seed, MZ_RNG_TIE, gid, step, ((uint32_t)sim << 12) | (uint32_t)depth);
                    ach = nth_set_bit(mask, (int)mz_rng_below(r, (uint32_t)nt));
                }
            }
            ncc = gor<GW>(a == ach ? nc : 0u);           // the chosen lane's nc, via DPP
        }
        const int ei = (int)__umul24((unsigned)e, (unsigned)A) + ach;
        const int Cch = (int)(ncc >> 16);
        const bool keep = a == depth;                     // depth < GW: lane `depth` keeps the level
        pe = keep ? ei : pe;
        pc = keep ? Cch - 1 : pc;
        if (depth >= GW && a == 0) { path[2 * depth] = ei; path[2 * depth + 1] = Cch - 1; }
        vtp = vtp >= players ? 1 : vtp + 1;             // mod1(vtp + 1, |players|), :267
        if (Cch == 0) { out = SelectOut{e, ach, vtp, depth}; break; }
        e = Cch - 1; Np = (int)(ncc & 0xffffu);
    }
    if (a >= 1 && a <= out.depth) { path[2 * a] = pe; path[2 * a + 1] = pc; }
    return out;
}

// ---------------------------------------------------------------------------
// Cached select (the small kernel, GW = 16).  select_child's argmax at a node
// depends on the node's N, its children's (N, W, P, ev) and MinMaxStats.  The
// first two change only when the node lies on a backup path; MinMaxStats
// changes with any backup.  So after every backup the argmax of each node on
// the path is recomputed (cache_row, all waves, one 16-lane row per node),
// and of EVERY expanded node when the backup moved min or max (the game's
// tag `ver` is then bumped).  An entry {ver << 5 | child, nc of that edge}
// stamped with the current tag is therefore exactly select_child's answer,
// and select walks the tree by one LDS read per level.  A node whose maximum
// ties is stored as 0 (never current): select computes it in full, with the
// Philox TIE draw keyed by (simulation, depth) as the oracle does.  The score
// is the same f32/f64 expression as select_path's, so the entries are
// bit-identical to a full evaluation.
// Lane-mask helpers (SGPR masks, no i1 round trips): v_cmp into an SGPR
// pair, and v_cndmask on one.
__device__ __forceinline__ uint64_t mz_vcmp_ne(uint32_t x, uint32_t y) {
    uint64_t m;
    asm("v_cmp_ne_u32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(y));
    return m;
}
__device__ __forceinline__ uint64_t mz_vcmp_eq(uint32_t x, uint32_t y) {
    uint64_t m;
    asm("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(y));
    return m;
}
__device__ __forceinline__ int mz_vsel(uint64_t m, int if_set, int if_clear) {
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
    return r;
}

// diagnostic (same results): MZ_DIAG_DIV_TWICE computes the pUCT normalisation and the backup's
// W / N quotients twice — are those divisions on the critical path?
__device__ __forceinline__ float mz_div_diag(float x, float y) {
#ifdef MZ_DIAG_DIV_TWICE
    float q0 = x / y;
    asm volatile("" : "+v"(x) : "v"(q0));
#endif
    return x / y;
}

__device__ __forceinline__ float pucb_score(const float4& ed, const double* prow, int Np, bool lg, bool norm,
                                            float mmin, float den) {
    const uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
    const int Nc = (int)(nc & 0xffffu);
    const double pb_c = prow[Nc < Np ? Nc : Np];
    const float vn = mz_div_diag(ed.w - mmin, den);
    const float vs = Nc > 0 ? (norm ? vn : ed.w) : 0.0f;
    const double prior_score = pb_c * (double)ed.z;
    const float us = (float)(prior_score + (double)vs);
    return lg ? us : -INFINITY;
}

// The same score without the pb_term table (select_path<false>: the pbc and
// sqrt entries of the parent and one f64 division; S too large for the triangle).
__device__ __forceinline__ float pucb_score_nt(const float4& ed, double pbn, double sqn, bool lg, bool norm,
                                               float mmin, float den) {
    const uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
    const int Nc = (int)(nc & 0xffffu);
    const double pb_c = pbn * (sqn / (double)(Nc + 1));
    const float vn = (ed.w - mmin) / den;
    const float vs = Nc > 0 ? (norm ? vn : ed.w) : 0.0f;
    const double prior_score = pb_c * (double)ed.z;
    const float us = (float)(prior_score + (double)vs);
    return lg ? us : -INFINITY;
}

// the score of this lane's child of node e (parent visits Np): with the
// pb_term triangle (TAB) or the pbc / sqrt tables
template <bool TAB>
__device__ __forceinline__ float pucb_lane(const float4& ed, int Np, bool lg, bool norm, float mmin, float den,
                                           const double* pbterm, const double* pbc_tab, const double* sqrt_tab) {
    if constexpr (TAB)
        return pucb_score(ed, pbterm + (__umul24((unsigned)Np, (unsigned)(Np + 1)) >> 1), Np, lg, norm, mmin, den);
    else
        return pucb_score_nt(ed, pbc_tab[Np], sqrt_tab[Np], lg, norm, mmin, den);
}

template <int GW> __device__ __forceinline__ float gmax_sel(float u) {
    if constexpr (GW == 16) return g16_vmax_to(u);
    else return gmax<GW>(u);
}
template <int GW> __device__ __forceinline__ uint32_t grp_mask(uint64_t m, int lane) {
    return (uint32_t)(m >> (lane & (64 - GW))) & (GW == 32 ? 0xffffffffu : 0xffffu);
}

// One GW-lane group (row-uniform call) recomputes node `slot`'s entry; with
// `cache_g` the entry is also stored there (the tree's HBM home).
template <int GW = 16, bool TAB = true>
__device__ __forceinline__ int cache_row(const TreeView& t, uint2* cache, uint32_t tag, int slot, int Np, bool lg,
                                         int a, int A, float mmin, float mmax, const double* pbterm, int lane,
                                         const double* pbc_tab = nullptr, const double* sqrt_tab = nullptr,
                                         uint2* cache_g = nullptr) {
    const int ac = a < A ? a : A - 1;
    const float4 ed = t.e[(int)__umul24((unsigned)slot, (unsigned)A) + ac];
    const float u = pucb_lane<TAB>(ed, Np, lg, mmax > mmin, mmin, mmax - mmin, pbterm, pbc_tab, sqrt_tab);
    const float m = gmax_sel<GW>(u);
    const uint32_t msk = grp_mask<GW>(__builtin_amdgcn_ballot_w64(lg && u == m), lane);
    const int ach = (int)__builtin_ctzll((uint64_t)msk | (1ull << GW));
    const bool tie = (msk & (msk - 1)) != 0;
    if (a == ach) {
        const uint2 v = tie ? make_uint2(0u, 0u) : make_uint2((tag << 5) | (uint32_t)ach, __builtin_bit_cast(uint32_t, ed.x));
        cache[slot] = v;
        if (cache_g) cache_g[slot] = v;
    }
    return tie ? -1 : ach;                               // the entry's child (-1: evaluated in full at select)
}

// U nodes at once (independent rows, one GW-lane group per game): every load
// of the U nodes is issued before any score is formed, so one pass costs about
// one node's latency.  Inactive entries (act = false, group-uniform) compute on
// slot 0 and store nothing.
template <int GW, bool TAB, int U>
__device__ __forceinline__ void cache_rows(const TreeView& t, uint2* cache, uint32_t tag, const int (&slot)[U],
                                           const int (&Np)[U], const bool (&act)[U], bool lg, int a, int A,
                                           float mmin, float mmax, const double* pbterm, int lane,
                                           const double* pbc_tab, const double* sqrt_tab, uint2* cache_g,
                                           int* ch_out = nullptr) {
    const int ac = a < A ? a : A - 1;
    float4 ed[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ed[u] = t.e[(int)__umul24((unsigned)(act[u] ? slot[u] : 0), (unsigned)A) + ac];
    float sc[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        sc[u] = pucb_lane<TAB>(ed[u], act[u] ? Np[u] : 0, lg, mmax > mmin, mmin, mmax - mmin, pbterm, pbc_tab,
                               sqrt_tab);
    float m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) m[u] = gmax_sel<GW>(sc[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t msk = grp_mask<GW>(__builtin_amdgcn_ballot_w64(lg && sc[u] == m[u]), lane);
        const int ach = (int)__builtin_ctzll((uint64_t)msk | (1ull << GW));
        if (ch_out) ch_out[u] = (msk & (msk - 1)) != 0 ? -1 : ach;   // the entry's child (-1: a tie)
        if (act[u] && a == ach) {
            const bool tie = (msk & (msk - 1)) != 0;
            const uint2 v = tie ? make_uint2(0u, 0u)
                                : make_uint2((tag << 5) | (uint32_t)ach, __builtin_bit_cast(uint32_t, ed[u].x));
            cache[slot[u]] = v;
            if (cache_g) cache_g[slot[u]] = v;
        }
    }
}

// select_path (TAB, GW = 16) with the per-node cache: a level whose entry
// carries the game's current tag costs one ds_read_b64 (the next slot and N
// come with it); otherwise (a tie, or the root before the first backup) the
// level is evaluated in full, behind one wave-uniform test.  The games of the
// wave walk in lockstep, so `depth` is wave-uniform; to_play at the leaf is
// mod1(root_tp + depth, |players|) (SelfPlay.jl:267), formed once.
template <int GW = 16, bool TAB = true>
__device__ __forceinline__ SelectOut select_path_cached(const TreeView& t, const uint2* cache, uint32_t ver,
                                                        int* path, int root_N, int root_tp, uint32_t legal,
                                                        float mmin, float mmax, int a, int lane, int A, int players,
                                                        const double* pbterm, uint64_t seed, uint32_t gid,
                                                        uint32_t step, int sim, const double* pbc_tab = nullptr,
                                                        const double* sqrt_tab = nullptr, int D = 0, int e0 = 0,
                                                        uint32_t npc0 = 0) {
    const bool lg = a < A && ((legal >> a) & 1u);
    const bool norm = mmax > mmin;
    const float den = mmax - mmin;
    const int ac = a < A ? a : A - 1;
    const uint64_t lgmask = __builtin_amdgcn_ballot_w64(lg);
    // Lane state, frozen per group once its leaf is reached: e = the node being
    // selected from (at the end: the leaf's parent), npc = the nc word of the
    // edge into e (its N), lach / dg = action and depth of the last level
    // walked.  `am` = lanes whose group is still walking (an SGPR mask, so the
    // freezes are single v_cndmask ops and the loop exit a scalar test).
    // Skip-ahead: a group starts at level D (its node e0, npc0 the nc word of
    // the edge into it): the recompute found levels 0..D-1 of the last path
    // still selected (their entries current and pointing along it), so the walk
    // from the root would retrace them; lv = the level being chosen, per group.
    int e = D > 0 ? e0 : 0, dg = D, lach = 0, pe = 0, pc = 0;
    uint32_t npc = D > 0 ? npc0 : (uint32_t)root_N;
    uint64_t am = __builtin_amdgcn_ballot_w64(true);
    // the next level's entry is read as soon as its node is known, before this
    // level's path bookkeeping, so the LDS latency runs under that bookkeeping
    uint2 cn = cache[e];
    for (int it = 1;; ++it) {
        const int lv = D + it;
        uint2 ce = cn;
        asm volatile("" : "+v"(ce.x), "+v"(ce.y));       // one ds_read_b64 (not split into the branches)
        int ach = (int)(ce.x & 31u);
        uint32_t ncc = ce.y;
        const uint64_t stm = mz_vcmp_ne(ce.x >> 5, ver) & am;
        if (stm != 0) {                                   // rare: the level in full, for every group
            const bool stale = (stm >> lane) & 1u;
            const int Np = (int)(npc & 0xffffu);
            const float4 ed = t.e[(int)__umul24((unsigned)e, (unsigned)A) + ac];
            const uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
            const float u = pucb_lane<TAB>(ed, Np, lg, norm, mmin, den, pbterm, pbc_tab, sqrt_tab);
            const float m = gmax_sel<GW>(u);
            uint64_t eqm;
            asm volatile("v_cmp_eq_f32_e64 %0, %1, %2" : "=s"(eqm) : "v"(u), "v"(m));
            const uint32_t mask = grp_mask<GW>(eqm & lgmask, lane);
            int ch = (int)__builtin_ctzll((uint64_t)mask | (1ull << GW));
            const int nt = __builtin_popcount(mask);
            if (stale && nt > 1) {                        // ties: the Philox draw (oracle select_child)
                const uint32_t r = mz_rng_u32(seed, MZ_RNG_TIE, gid, step, ((uint32_t)sim << 12) | (uint32_t)lv);
                ch = nth_set_bit(mask, (int)mz_rng_below(r, (uint32_t)nt));
            }
            const uint32_t nch = gor<GW>(a == ch ? nc : 0u);
            ach = stale ? ch : ach;
            ncc = stale ? nch : ncc;
        }
        const int ei = (int)__umul24((unsigned)e, (unsigned)A) + ach;
        const int Cch = (int)(ncc >> 16);                 // child slot + 1, 0 = the leaf
        const uint64_t nm = mz_vcmp_ne((uint32_t)Cch, 0u) & am;   // groups still walking after this level
        const int en = mz_vsel(nm, Cch - 1, e);
        cn = cache[en];                                   // (a frozen group re-reads its own node: harmless)
        const uint64_t km = mz_vcmp_eq((uint32_t)a, (uint32_t)lv) & am;   // lane `lv` keeps the level
        pe = mz_vsel(km, ei, pe);
        pc = mz_vsel(km, Cch, pc);
        lach = mz_vsel(am, ach, lach);
        dg = mz_vsel(am, lv, dg);
        const uint64_t deep = __builtin_amdgcn_ballot_w64(lv >= GW) & am;
        if (deep != 0) {                                  // rare: deep paths past the register-held levels
            uint64_t wm = deep;
            asm volatile("" : "+s"(wm));                  // the lane test stays inside this branch
            if (a == 0 && ((wm >> lane) & 1u)) { path[2 * lv] = ei; path[2 * lv + 1] = Cch - 1; }
        }
        e = en;
        npc = (uint32_t)mz_vsel(nm, (int)ncc, (int)npc);
        am = nm;
        if (am == 0) break;
    }
    if (a > D && a <= dg && a < GW) { path[2 * a] = pe; path[2 * a + 1] = pc - 1; }
    const int vtp = players == 2 ? ((root_tp - 1 + dg) & 1) + 1 : (root_tp - 1 + dg) % players + 1;
    return SelectOut{e, lach, vtp, dg};
}

// backpropagate! (SelfPlay.jl:190-217), quirk Q7, for the GW-lane group.
// Node d of the path (0 = root ... depth = the just-expanded leaf with
// to_play tl) receives v_in(d): v_in(depth) = the leaf value; otherwise
// v_in(d) = v_out(d+1) with v_out(k) = (tp_k == tl) ? -R_k : R_k + γ v_in(k).
// v_out resets wherever tp_k == tl, so every level's v_in is the same f32
// expression chain the sequential loop evaluates, started at the nearest
// reset below it (one or two levels away in 2-player games, where to_play
// alternates with depth): all levels update in parallel, bit-exactly.  The
// min-max fold is order-independent (exact comparisons).  1-player games
// have no resets and run the sequential loop on lane 0.
template <int GW = 16>
__device__ __forceinline__ void backup_path(const TreeView& t, const int* path, int depth, float value, int tl,
                                            int A, int players, float discount, int& root_N, float& root_W,
                                            int root_tp, float& mmin, float& mmax, int a, uint2* lvl = nullptr,
                                            int* nN = nullptr) {
    if (players != 2) {
        if (a == 0) {
            float v = value;
            for (int d = depth; d >= 0; --d) {
                int N; float W, R; int i = 0;
                uint32_t nc = 0;
                if (d > 0) {
                    i = path[2 * d]; nc = t.nc(i);
                    N = (int)(nc & 0xffffu); W = t.w(i); R = t.nr[path[2 * d + 1]];
                } else {
                    N = root_N; W = root_W; R = 0.0f;
                }
                W = W + v; N += 1;
                const float q = W / (float)N;
                const float upd = R + discount * q;
                mmin = mmin < upd ? mmin : upd; mmax = mmax > upd ? mmax : upd;
                v = R + discount * v;
                if (d > 0) {
                    t.nc(i) = (nc & 0xffff0000u) | (uint32_t)N; t.w(i) = W;
                    t.ev(i) = R + (players == 1 ? discount * q : discount * (-q));
                }
                else { root_N = N; root_W = W; }
                if (lvl) {                               // the cached select's (slot, N) per level
                    const int c = d > 0 ? path[2 * d + 1] : 0;
                    lvl[d] = make_uint2((uint32_t)c, (uint32_t)N); nN[c] = N;
                }
            }
        }
        root_N = __shfl(root_N, 0, GW); root_W = __shfl(root_W, 0, GW);
        mmin = __shfl(mmin, 0, GW); mmax = __shfl(mmax, 0, GW);
        return;
    }
    // two players: to_play alternates with depth (node k has mod1(root_tp + k),
    // the virtual_to_play of SelfPlay.jl:267), so below level d < depth the
    // nearest reset is k0 = d+1 if tp(d+1) == tl, else d+2 (the leaf, level
    // depth, always resets): v_in(d) = -R(d+1) or R(d+1) + γ(-R(d+2)).  Each
    // lane issues its reads in two round trips: path entries of d, d+1, d+2,
    // then the edge record and the children's R / to_play.
    float lmin = INFINITY, lmax = -INFINITY;
    int rN = root_N; float rW = root_W;
    for (int base = 0; base <= depth; base += GW) {
        const int d = base + a;
        if (d <= depth) {
            const int i = d > 0 ? path[2 * d] : 0;
            const int c = d > 0 ? path[2 * d + 1] : 0;
            const int c1 = d + 1 <= depth ? path[2 * d + 3] : 0;
            const int c2 = d + 2 <= depth ? path[2 * d + 5] : 0;
            const float4 ed = t.e[i];
            const float Rc = t.nr[c];
            const int tpc = t.ntp[c];
            const float R1 = t.nr[c1], R2 = t.nr[c2];
            const int tp1 = t.ntp[c1];
            uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
            int N; float W, R; int tp;
            if (d > 0) { N = (int)(nc & 0xffffu); W = ed.y; R = Rc; tp = tpc; }
            else { N = root_N; W = root_W; R = 0.0f; tp = root_tp; }
            float vin;
            if (d == depth) vin = value;
            else if (tp1 == tl) vin = -R1;
            else vin = R1 + discount * (-R2);
            W = tp == tl ? W + vin : W - vin;
            N += 1;
            const float q = W / (float)N;
            const float upd = R + discount * q;
            lmin = lmin < upd ? lmin : upd;
            lmax = lmax > upd ? lmax : upd;
            if (d > 0) {
                nc = (nc & 0xffff0000u) | (uint32_t)N;
                t.nc(i) = nc; t.w(i) = W; t.ev(i) = R + discount * (-q);
            } else { rN = N; rW = W; }
            if (lvl) { lvl[d] = make_uint2((uint32_t)c, (uint32_t)N); nN[c] = N; }   // the cached select's (slot, N)
        }
    }
    lmin = gmin<GW>(lmin);
    lmax = gmax<GW>(lmax);
    mmin = mmin < lmin ? mmin : lmin;
    mmax = mmax > lmax ? mmax : lmax;
    // lane 0 of the group (level 0 = the root) to all GW lanes: DPP row broadcast
    if constexpr (GW == 16) {
        root_N = __builtin_amdgcn_update_dpp(0, rN, 0x150, 0xF, 0xF, false);
        root_W = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, rW), 0x150, 0xF, 0xF, false));
    } else {
        root_N = __shfl(rN, 0, GW); root_W = __shfl(rW, 0, GW);
    }
}

// The two-player backup of the small kernels with its loads issued early:
// backup_preload reads lane d's path entries, edge record and the children's
// reward / to_play for the first GW levels BEFORE the read-out activations
// (the f64 tanh chains) and before the leaf's expansion writes (the child
// link of the leaf edge, the new slot's reward / to_play, path[2·depth+1]);
// backup_path_pre then patches exactly those values in registers (the new slot
// e_new is referenced only by the leaf level: a fresh slot no older path entry
// points to) and runs backup_path's arithmetic, in the same order, on them.
// Same loads and stores as the caller's writes + backup_path, so the same bits;
// the LDS round trips overlap the read-outs.  Deep paths (depth >= GW) run the
// levels past the first block as backup_path does, after the writes.
struct BackupPre {
    int i, c, c1, c2, tpc, tp1;
    float4 ed;
    float Rc, R1, R2;
};
template <int GW = 16>
__device__ __forceinline__ BackupPre backup_preload(const TreeView& t, const int* path, int depth, int a) {
    BackupPre b;
    const int d = a < GW ? a : 0;
    b.i = d > 0 && d <= depth ? path[2 * d] : 0;
    b.c = d > 0 && d < depth ? path[2 * d + 1] : 0;
    b.c1 = d + 1 < depth ? path[2 * d + 3] : 0;
    b.c2 = d + 2 < depth ? path[2 * d + 5] : 0;
    b.ed = t.e[b.i];
    b.Rc = t.nr[b.c]; b.tpc = t.ntp[b.c];
    b.R1 = t.nr[b.c1]; b.tp1 = t.ntp[b.c1];
    b.R2 = t.nr[b.c2];
    return b;
}
template <int GW = 16>
__device__ __forceinline__ void backup_path_pre(const TreeView& t, const int* path, BackupPre b, int depth, float value,
                                                float rew, int e_new, int tl, float discount, int& root_N,
                                                float& root_W, int root_tp, float& mmin, float& mmax, int a,
                                                uint2* lvl, int* nN) {
    float lmin = INFINITY, lmax = -INFINITY;
    int rN = root_N; float rW = root_W;
    {
        const int d = a;
        if (d <= depth && d < GW) {
            // the leaf's expansion, as the caller has just written it
            if (d == depth && d > 0) {
                b.c = e_new; b.Rc = rew; b.tpc = tl;
                b.ed.x = __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, b.ed.x) & 0xffffu) |
                                                   ((uint32_t)(e_new + 1) << 16));
            }
            if (d + 1 == depth) { b.c1 = e_new; b.R1 = rew; b.tp1 = tl; }
            if (d + 2 == depth) { b.c2 = e_new; b.R2 = rew; }
            uint32_t nc = __builtin_bit_cast(uint32_t, b.ed.x);
            int N; float W, R; int tp;
            if (d > 0) { N = (int)(nc & 0xffffu); W = b.ed.y; R = b.Rc; tp = b.tpc; }
            else { N = root_N; W = root_W; R = 0.0f; tp = root_tp; }
            float vin;
            if (d == depth) vin = value;
            else if (b.tp1 == tl) vin = -b.R1;
            else vin = b.R1 + discount * (-b.R2);
            W = tp == tl ? W + vin : W - vin;
            N += 1;
            const float q = mz_div_diag(W, (float)N);
            const float upd = R + discount * q;
            lmin = lmin < upd ? lmin : upd;
            lmax = lmax > upd ? lmax : upd;
            if (d > 0) {
                nc = (nc & 0xffff0000u) | (uint32_t)N;
                t.nc(b.i) = nc; t.w(b.i) = W; t.ev(b.i) = R + discount * (-q);
            } else { rN = N; rW = W; }
            lvl[d] = make_uint2((uint32_t)b.c, (uint32_t)N); nN[b.c] = N;
        }
    }
    for (int base = GW; base <= depth; base += GW) {        // deep paths: backup_path's loop
        const int d = base + a;
        if (d <= depth) {
            const int i = path[2 * d];
            const int c = path[2 * d + 1];
            const int c1 = d + 1 <= depth ? path[2 * d + 3] : 0;
            const int c2 = d + 2 <= depth ? path[2 * d + 5] : 0;
            const float4 ed = t.e[i];
            const float Rc = t.nr[c];
            const int tpc = t.ntp[c];
            const float R1 = t.nr[c1], R2 = t.nr[c2];
            const int tp1 = t.ntp[c1];
            uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
            int N = (int)(nc & 0xffffu); float W = ed.y;
            float vin;
            if (d == depth) vin = value;
            else if (tp1 == tl) vin = -R1;
            else vin = R1 + discount * (-R2);
            W = tpc == tl ? W + vin : W - vin;
            N += 1;
            const float q = W / (float)N;
            const float upd = Rc + discount * q;
            lmin = lmin < upd ? lmin : upd;
            lmax = lmax > upd ? lmax : upd;
            nc = (nc & 0xffff0000u) | (uint32_t)N;
            t.nc(i) = nc; t.w(i) = W; t.ev(i) = Rc + discount * (-q);
            lvl[d] = make_uint2((uint32_t)c, (uint32_t)N); nN[c] = N;
        }
    }
    lmin = gmin<GW>(lmin);
    lmax = gmax<GW>(lmax);
    mmin = mmin < lmin ? mmin : lmin;
    mmax = mmax > lmax ? mmax : lmax;
    if constexpr (GW == 16) {
        root_N = __builtin_amdgcn_update_dpp(0, rN, 0x150, 0xF, 0xF, false);
        root_W = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, rW), 0x150, 0xF, 0xF, false));
    } else {
        root_N = __shfl(rN, 0, GW); root_W = __shfl(rW, 0, GW);
    }
}

// backpropagate! (SelfPlay.jl:190-217) for 1-player games, lane-parallel.
// Without to_play resets the incoming value is the linear chain v_in(depth)
// = leaf value, v_in(d-1) = R_d + γ·v_in(d), which the sequential loop
// evaluates node by node.  Here the lanes first stage R_d (node d's reward)
// in `rr`, every lane runs the same f32 chain over the staged values (two
// ops per level, no memory on the critical path; round 5: GW rewards per LDS
// wait and v_in kept in registers, +0.7 % on configs[4], tools/gpu_r05y.sh)
// and stores v_in(d) in `vin`; then each lane updates its own levels as the
// sequential loop would (W + v, N + 1, q = W/N, R + γq).  Same f32 operations, same results;
// `rr`/`vin` hold depth + 1 floats (LDS, this group's own).
template <int GW>
__device__ __forceinline__ void backup_path_1p(const TreeView& t, const int* path, int depth, float value,
                                               float discount, int& root_N, float& root_W, float& mmin,
                                               float& mmax, int a, float* rr, float* vin, uint2* lvl = nullptr,
                                               int* nN = nullptr) {
    for (int d = 1 + a; d <= depth; d += GW) rr[d] = t.nr[path[2 * d + 1]];
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    float v = value;
    // GW levels per LDS wait: the group's staged rewards of levels cGW ..
    // cGW+GW-1 as one broadcast batch, the chain over registers, lane l
    // keeping v_in(cGW + l) by a select beside the chain (one store per batch
    // instead of one per level).  Levels outside 1..depth leave v as it is.
    for (int c = depth / GW; c >= 0; --c) {
        float r[GW];
        const float4* r4 = reinterpret_cast<const float4*>(rr + c * GW);
#pragma unroll
        for (int q = 0; q < GW / 4; ++q) {
            const float4 x = r4[q];
            r[4 * q] = x.x; r[4 * q + 1] = x.y; r[4 * q + 2] = x.z; r[4 * q + 3] = x.w;
        }
        float mine = v;
#pragma unroll
        for (int l = GW - 1; l >= 0; --l) {
            const int lv = c * GW + l;
            mine = a == l ? v : mine;                 // v_in(lv)
            const float nv = r[l] + discount * v;
            v = lv >= 1 && lv <= depth ? nv : v;
        }
        if (c * GW + a <= depth) vin[c * GW + a] = mine;
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    float lmin = INFINITY, lmax = -INFINITY;
    int rN = root_N; float rW = root_W;
    for (int d0 = a; d0 <= depth; d0 += GW) {
        const int i = d0 > 0 ? path[2 * d0] : 0;
        const float4 ed = t.e[i];
        const float vi = vin[d0];
        uint32_t nc = __builtin_bit_cast(uint32_t, ed.x);
        int N; float W, R;
        if (d0 > 0) { N = (int)(nc & 0xffffu); W = ed.y; R = rr[d0]; }
        else { N = root_N; W = root_W; R = 0.0f; }
        W = W + vi; N += 1;
        const float q = W / (float)N;
        const float upd = R + discount * q;
        lmin = lmin < upd ? lmin : upd;
        lmax = lmax > upd ? lmax : upd;
        if (d0 > 0) {
            nc = (nc & 0xffff0000u) | (uint32_t)N;
            t.nc(i) = nc; t.w(i) = W; t.ev(i) = R + discount * q;
        } else { rN = N; rW = W; }
        if (lvl) {                                       // the cached select's (slot, N) per level
            const int c = d0 > 0 ? path[2 * d0 + 1] : 0;
            lvl[d0] = make_uint2((uint32_t)c, (uint32_t)N); nN[c] = N;
        }
    }
    lmin = gmin<GW>(lmin);
    lmax = gmax<GW>(lmax);
    mmin = mmin < lmin ? mmin : lmin;
    mmax = mmax > lmax ? mmax : lmax;
    root_N = __shfl(rN, 0, GW); root_W = __shfl(rW, 0, GW);
}

// select_action (SelfPlay.jl:293-306) for a GW-lane group, called by every
// lane of the group with its own child's count Nc (lane a = action a): the
// oracle's rule (legal actions in ascending order).  The N^(1/T) weights are
// computed lane-parallel; the ordered scans read the lanes by shuffle with
// static indices, so nothing lands in a scratch frame.  Every lane returns
// the action.
template <int GW>
__device__ __forceinline__ int select_action_dev(int Nc, uint32_t legal, int A, float temperature, uint32_t r) {
    const int a = (int)(threadIdx.x % GW);
    legal &= A >= 32 ? 0xffffffffu : (1u << A) - 1u;
    const bool lg = (legal >> a) & 1u;
    const int n = __builtin_popcount(legal);
    const int last = 31 - __builtin_clz(legal);
    if (isinf(temperature)) return nth_set_bit(legal, (int)mz_rng_below(r, (uint32_t)n));
    // the weight each lane contributes: N (T = 0 and T = 1) or f32(N^(1/T))
    const bool gen = temperature != 0.0f && temperature != 1.0f;
    const float wl = gen ? (lg && Nc > 0 ? (float)det_exp(det_log((double)Nc) * (double)(1.0f / temperature)) : 0.0f)
                         : 0.0f;
    const int c = lg ? Nc : 0;
    if (temperature == 0.0f) {                        // argmax, the first maximum
        int best = -1, bc = 0;
#pragma unroll
        for (int b = 0; b < GW; ++b) {
            const int cb = __shfl(c, b, GW);
            if (((legal >> b) & 1u) && (best < 0 || cb > bc)) { best = b; bc = cb; }
        }
        return best;
    }
    if (!gen) {                                       // T = 1: ∝ N, the integer counts exactly
        uint32_t tot = 0;
#pragma unroll
        for (int b = 0; b < GW; ++b) tot += (uint32_t)__shfl(c, b, GW);
        if (tot == 0) return nth_set_bit(legal, (int)mz_rng_below(r, (uint32_t)n));
        const uint32_t tt = mz_rng_below(r, tot);
        uint32_t cum = 0;
        int pick = -1;
#pragma unroll
        for (int b = 0; b < GW; ++b) {
            cum += (uint32_t)__shfl(c, b, GW);
            if (((legal >> b) & 1u) && pick < 0 && cum > tt) pick = b;
        }
        return pick >= 0 ? pick : last;
    }
    float s = 0.0f;                                   // ∝ N^(1/T): f32 sum in ascending order
#pragma unroll
    for (int b = 0; b < GW; ++b) {
        const float wb = __shfl(wl, b, GW);
        if ((legal >> b) & 1u) s = s + wb;
    }
    const float u = (float)(r >> 8) * 5.9604644775390625e-08f * s;
    float cum = 0.0f;
    int pick = -1;
#pragma unroll
    for (int b = 0; b < GW; ++b) {
        const float wb = __shfl(wl, b, GW);
        if (((legal >> b) & 1u) && pick < 0) { cum = cum + wb; if (cum > u) pick = b; }
    }
    return pick >= 0 ? pick : last;
}

// Copy one game's tree to the global debug buffers (parity tests only).
template <int GW = 16>
__device__ __forceinline__ void dump_tree(const TreeView& t, const TreeView& dst, int n_edges, int n_nodes,
                                          int lane) {
    for (int i = lane; i < n_edges; i += GW) dst.e[i] = t.e[i];
    for (int i = lane; i < n_nodes; i += GW) { dst.nr[i] = t.nr[i]; dst.ntp[i] = t.ntp[i]; }
}
