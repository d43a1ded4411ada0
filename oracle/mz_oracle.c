/*
 * mz_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of deveshjawla/MuZero.jl's hot path in its
 * documented `ref_semantics` (SURVEY.md §2.1, quirks Q1–Q17), used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product (libmz) never links, loads or calls it.
 *
 * PARITY UNPINNED: the reference is Julia-only and Julia is absent from this
 * image and the GPU box, and the reference ships no tests,
 * fixtures or golden vectors.  This restatement is therefore checked by an
 * independent Python mirror written from the Julia source
 * (tests/mirror_ref.py) and the networks against torch-CPU fp32 autograd-free
 * forwards; golden vectors under tests/golden/ are generated from it by
 * tests/golden/make_golden.py.
 *
 * Contract decisions where the reference is not reproducible (Q6) or its
 * third-party arithmetic is unavailable (Flux/NNlib/Distributions):
 *   - RNG: Philox4x32-10 streams (include/mz_detmath.h) replace Julia's
 *     global unseeded RNG and MersenneTwister(1234);
 *   - children are visited in ascending action order (reference: Dict order);
 *   - Dense dot products use the canonical order of mz_dot below;
 *   - exp/tanh/log are the deterministic det_* functions.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mz.h"
#include "../include/mz_detmath.h"

#define EXPORT __attribute__((visibility("default")))
#define MAXA MZ_MAX_ACTIONS

/* ===================================================================== nets
 * Learning.jl:70-142 (FeedForwardHP) and 148-255 (ResNetHP, the intended
 * architecture of SURVEY §2.1 Q12 / DESIGN.md §9).  Layer list of each net
 * in Flux.params order: Dense W (out,in) col-major then b; Conv weight
 * (kw,kh,cin,cout) col-major then b; BatchNorm β then γ (its running μ = 0,
 * σ² = 1 are state, not params, and the reference's test-mode forward never
 * changes them).                                                           */
typedef struct { int32_t kind; mz_ffhp ff; mz_resnet_hp rn; } ora_nethp;   /* kind 0 FC, 1 ResNet */

typedef struct {
    int in, out, act;          /* Dense: features; Conv: channels */
    size_t woff, boff;
    int conv, kw, kh, pw, ph, W, H;   /* Conv (zero pad, kernel flipped); output board W x H */
    int sw, sh, Wi, Hi;        /* stride and input board (stride 1: Wi x Hi = W x H) */
    int pool;                  /* MeanPool(kw x kh, stride, pad) of `in` = `out` channels, no params */
    int bn; size_t bnoff;      /* BatchNorm(out) after the affine: β at bnoff, γ at bnoff + out */
    int res_save, res_add;     /* block input saved here / added before the activation */
} OLayer;
typedef struct {
    int n[3];            /* layers in trunk, head 1, head 2 (head counts 0 for repr) */
    OLayer L[3][96];
    size_t nparams;
    int softmax_head2;   /* prediction policy head ends in softmax (Learning.jl:113-114) */
    int maxact;          /* largest activation (floats) */
} ONet;

static int olayer_insize(const OLayer* l) { return l->conv ? l->in * l->Wi * l->Hi : l->in; }
static int olayer_outsize(const OLayer* l) { return l->conv ? l->out * l->W * l->H : l->out; }

static OLayer* onet_add(ONet* net, int part, int in, int out, int act) {
    OLayer* l = &net->L[part][net->n[part]++];
    memset(l, 0, sizeof(*l));
    l->in = in; l->out = out; l->act = act;
    l->woff = net->nparams; net->nparams += (size_t)in * out;
    l->boff = net->nparams; net->nparams += (size_t)out;
    return l;
}

/* make_dense (Learning.jl:70-78): Dense(in, out, relu), or with
 * use_batch_norm Chain(Dense(in, out), BatchNorm(out, relu)) — β, γ follow
 * the Dense's W, b in Flux.params */
static OLayer* onet_dense(ONet* net, int part, int in, int out, int bn) {
    OLayer* l = onet_add(net, part, in, out, MZ_ACT_RELU);
    if (bn) { l->bn = 1; l->bnoff = net->nparams; net->nparams += (size_t)2 * out; }
    return l;
}

/* Conv(k, in => out, pad = k .÷ 2) [+ BatchNorm(out, act)] on a W x H board */
static OLayer* onet_conv(ONet* net, int part, int in, int out, int kw, int kh, int W, int H, int bn, int act) {
    OLayer* l = &net->L[part][net->n[part]++];
    memset(l, 0, sizeof(*l));
    l->conv = 1; l->in = in; l->out = out; l->act = act;
    l->kw = kw; l->kh = kh; l->pw = kw / 2; l->ph = kh / 2; l->W = W; l->H = H;
    l->sw = 1; l->sh = 1; l->Wi = W; l->Hi = H;
    l->woff = net->nparams; net->nparams += (size_t)kw * kh * in * out;
    l->boff = net->nparams; net->nparams += (size_t)out;
    if (bn) { l->bn = 1; l->bnoff = net->nparams; net->nparams += (size_t)2 * out; }
    return l;
}

/* resnet_block (Learning.jl:148-158): conv-BN-relu-conv-BN, + x, relu */
static void onet_resblock(ONet* net, int part, int n, int k, int W, int H) {
    OLayer* a = onet_conv(net, part, n, n, k, k, W, H, 1, MZ_ACT_RELU);
    a->res_save = 1;
    OLayer* b = onet_conv(net, part, n, n, k, k, W, H, 1, MZ_ACT_RELU);
    b->res_add = 1;
}

/* Conv(k, in => out, stride = 2, pad = k .÷ 2) without BatchNorm or
 * activation (the downsampler's strided convs, Learning.jl:177,179) from a
 * Wi x Hi board to ((Wi + 2pw - kw) ÷ 2 + 1) x (...) */
static OLayer* onet_conv_s2(ONet* net, int in, int out, int kw, int kh, int Wi, int Hi) {
    const int W = (Wi + 2 * (kw / 2) - kw) / 2 + 1, H = (Hi + 2 * (kh / 2) - kh) / 2 + 1;
    OLayer* l = onet_conv(net, 0, in, out, kw, kh, W, H, 0, MZ_ACT_IDENTITY);
    l->sw = 2; l->sh = 2; l->Wi = Wi; l->Hi = Hi;
    return l;
}

/* MeanPool((3,3), stride = 2, pad = 1) (Learning.jl:181,183; the reference
 * writes MeanPool(3, ...), which Flux 0.12 only accepts as a tuple) */
static void onet_meanpool(ONet* net, int ch, int Wi, int Hi) {
    OLayer* l = &net->L[0][net->n[0]++];
    memset(l, 0, sizeof(*l));
    l->conv = 1; l->pool = 1; l->in = ch; l->out = ch; l->act = MZ_ACT_IDENTITY;
    l->kw = 3; l->kh = 3; l->pw = 1; l->ph = 1; l->sw = 2; l->sh = 2; l->Wi = Wi; l->Hi = Hi;
    l->W = (Wi + 2 - 3) / 2 + 1; l->H = (Hi + 2 - 3) / 2 + 1;
}

/* Board of the hidden state: the observation board, or with ResNetHP
 * downsample the board after the downsampler (two stride-2 convs and two
 * stride-2 pools: 84 -> 42 -> 21 -> 11 -> 6), which the reference computes
 * as representation_output_size (Learning.jl:173, taken from the wrong chain,
 * Q12) and prediction / dynamics read (:194, :229). */
static void rn_board(const mz_config* c, const mz_resnet_hp* hp, int* W, int* H) {
    int w = c->observation_shape[0], h = c->observation_shape[1];
    if (hp->downsample) {
        const int kw = hp->conv_kernel_size[0], kh = hp->conv_kernel_size[1];
        for (int i = 0; i < 2; ++i) { w = (w + 2 * (kw / 2) - kw) / 2 + 1; h = (h + 2 * (kh / 2) - kh) / 2 + 1; }
        for (int i = 0; i < 2; ++i) { w = (w + 2 - 3) / 2 + 1; h = (h + 2 - 3) / 2 + 1; }
    }
    *W = w; *H = h;
}

static int nethp_hidden(const mz_config* c, const ora_nethp* hp) {
    if (hp->kind == 0) return hp->ff.hidden_state_size;
    int W, H; rn_board(c, &hp->rn, &W, &H);
    return W * H * hp->rn.num_filters;
}

/* plane of the dynamics action input: the hidden state's board */
static int hid_plane(const mz_config* c, const ora_nethp* hp) {
    if (hp->kind == 0) return c->observation_shape[0] * c->observation_shape[1];
    int W, H; rn_board(c, &hp->rn, &W, &H);
    return W * H;
}

static void onet_finish(ONet* net) {
    net->maxact = 0;
    for (int p = 0; p < 3; ++p)
        for (int i = 0; i < net->n[p]; ++i) {
            const OLayer* l = &net->L[p][i];
            if (olayer_insize(l) > net->maxact) net->maxact = olayer_insize(l);
            if (olayer_outsize(l) > net->maxact) net->maxact = olayer_outsize(l);
        }
}

/* init_representation / init_prediction / init_dynamics for ResNetHP */
static void onet_build_resnet(ONet* net, int which, const mz_config* c, const mz_resnet_hp* hp) {
    int W, H, C = c->observation_shape[2];
    rn_board(c, hp, &W, &H);
    int nf = hp->num_filters, nb = hp->num_blocks, hs = hp->width_hidden, A = c->action_space_size;
    int P = W * H, nvf = hp->num_first_head_filters, npf = hp->num_second_head_filters;
    if (which == MZ_NET_REPR) {                                           /* :160-191 */
        int cin = C * (c->stacked_observations + 1) + c->stacked_observations;   /* Q12: the stacked input */
        int kw = hp->conv_kernel_size[0], kh = hp->conv_kernel_size[1];
        if (hp->downsample) {                                             /* :175-187 */
            /* `size` (undefined there) read as conv_kernel_size; indim[3] as
             * the stacked input's channels cin */
            int w = c->observation_shape[0], h = c->observation_shape[1];
            OLayer* l = onet_conv_s2(net, cin, cin, kw, kh, w, h);        /* :177 */
            w = l->W; h = l->H;
            for (int i = 0; i < 2; ++i) onet_resblock(net, 0, cin, kw, w, h);
            l = onet_conv_s2(net, cin, 2 * cin, kw, kh, w, h);            /* :179 */
            w = l->W; h = l->H;
            for (int i = 0; i < 3; ++i) onet_resblock(net, 0, 2 * cin, kw, w, h);
            onet_meanpool(net, 2 * cin, w, h);                            /* :181 */
            w = net->L[0][net->n[0] - 1].W; h = net->L[0][net->n[0] - 1].H;
            for (int i = 0; i < 3; ++i) onet_resblock(net, 0, 2 * cin, kw, w, h);
            onet_meanpool(net, 2 * cin, w, h);                            /* :183 */
            cin = 2 * cin;                                                /* :184: Conv(ksize, 2C => nf) */
        }
        onet_conv(net, 0, cin, nf, kw, kh, W, H, 1, MZ_ACT_RELU);
        for (int i = 0; i < nb; ++i) onet_resblock(net, 0, nf, kw, W, H);
    } else if (which == MZ_NET_PRED) {                                    /* :193-226 */
        onet_conv(net, 0, nf, nf, 1, 1, W, H, 1, MZ_ACT_RELU);
        for (int i = 0; i < nb; ++i) onet_resblock(net, 0, nf, 1, W, H);
        onet_conv(net, 1, nf, nvf, 1, 1, W, H, 1, MZ_ACT_RELU);           /* value head */
        onet_add(net, 1, P * nvf, hs, MZ_ACT_RELU);
        for (int i = 0; i < hp->depth_value; ++i) onet_add(net, 1, hs, hs, MZ_ACT_RELU);
        onet_add(net, 1, hs, 1, MZ_ACT_TANH);
        onet_conv(net, 2, nf, npf, 1, 1, W, H, 1, MZ_ACT_RELU);           /* policy head */
        onet_add(net, 2, P * npf, hs, MZ_ACT_IDENTITY);
        for (int i = 0; i < hp->depth_value; ++i) onet_add(net, 2, hs, hs, MZ_ACT_RELU);   /* :222 depth_value */
        onet_add(net, 2, hs, A, MZ_ACT_IDENTITY);
        net->softmax_head2 = 1;
    } else {                                                              /* :228-255 */
        onet_conv(net, 0, nf + 1, nf, 1, 1, W, H, 1, MZ_ACT_RELU);        /* Q12: + the one action plane */
        for (int i = 0; i < nb; ++i) onet_resblock(net, 0, nf, 1, W, H);
        onet_conv(net, 1, nf, nf, 1, 1, W, H, 1, MZ_ACT_RELU);            /* state head */
        for (int i = 0; i < nb; ++i) onet_resblock(net, 1, nf, 1, W, H);
        onet_conv(net, 2, nf, nvf, 1, 1, W, H, 1, MZ_ACT_RELU);           /* reward head */
        onet_add(net, 2, P * nvf, hs, MZ_ACT_RELU);
        for (int i = 0; i < hp->depth_value; ++i) onet_add(net, 2, hs, hs, MZ_ACT_RELU);
        onet_add(net, 2, hs, 1, hp->reward_activation);
    }
}

/* init_representation (Learning.jl:87-98) / init_prediction (:100-116) /
 * init_dynamics (:118-142) for FeedForwardHP. */
static void onet_build(ONet* net, int which, const mz_config* c, const ora_nethp* nh) {
    memset(net, 0, sizeof(*net));
    if (nh->kind == 1) { onet_build_resnet(net, which, c, &nh->rn); onet_finish(net); return; }
    const mz_ffhp* hp = &nh->ff;
    int W = c->observation_shape[0], H = c->observation_shape[1], C = c->observation_shape[2];
    int hs = hp->width_hidden, hid = hp->hidden_state_size, A = c->action_space_size;
    const int bn = hp->use_batch_norm != 0;
    if (which == MZ_NET_REPR) {
        int indim = W * H * (C * (c->stacked_observations + 1) + c->stacked_observations); /* :88 */
        onet_dense(net, 0, indim, hs, bn);
        for (int i = 0; i < hp->depth_representation; ++i) onet_dense(net, 0, hs, hs, bn);
        onet_add(net, 0, hs, hid, MZ_ACT_IDENTITY);
    } else if (which == MZ_NET_PRED) {
        onet_dense(net, 0, hid, hs, bn);
        for (int i = 0; i < hp->depth_prediction; ++i) onet_dense(net, 0, hs, hs, bn);
        for (int i = 0; i < hp->depth_value; ++i) onet_dense(net, 1, hs, hs, bn);
        onet_add(net, 1, hs, 1, MZ_ACT_TANH);                                  /* :110 */
        for (int i = 0; i < hp->depth_policy; ++i) onet_dense(net, 2, hs, hs, bn);
        onet_add(net, 2, hs, A, MZ_ACT_IDENTITY);                              /* :113 */
        net->softmax_head2 = 1;                                                 /* :114 */
    } else {
        int indim = W * H * (C + 1);                                            /* :120 */
        onet_dense(net, 0, indim, hs, bn);
        for (int i = 0; i < hp->depth_dynamics; ++i) onet_dense(net, 0, hs, hs, bn);
        for (int i = 0; i < hp->depth_state_head; ++i) onet_dense(net, 1, hs, hs, bn);
        onet_add(net, 1, hs, hid, MZ_ACT_IDENTITY);                            /* :136 */
        for (int i = 0; i < hp->depth_reward; ++i) onet_dense(net, 2, hs, hs, bn);
        onet_add(net, 2, hs, 1, hp->reward_activation);                        /* :140 */
    }
    onet_finish(net);
}

/* Canonical dot product of the engine: four partial fmaf chains over
 * contiguous k-quarters of length kq = 4*ceil(K/16), each started at +0,
 * combined as ((p0+p1)+(p2+p3)).  Flux's `W*x` (BLAS) has no fixed order;
 * this one is what the GPU's four-accumulator f32 MFMA chain computes.
 * Element k of output o's weight row is w[o*so + k*sk].                   */
static float mz_dot_s(const float* w, size_t sk, const float* x, int in) {
    int kq = 4 * ((in + 15) / 16);
    float p[4];
    for (int q = 0; q < 4; ++q) {
        p[q] = 0.0f;
        int k1 = (q + 1) * kq < in ? (q + 1) * kq : in;
        for (int k = q * kq; k < k1; ++k) p[q] = fmaf(w[(size_t)k * sk], x[k], p[q]);
    }
    return (p[0] + p[1]) + (p[2] + p[3]);
}
static float mz_dot(const float* Wcol /* W(out,in) col-major */, int out, int in, int o, const float* x) {
    return mz_dot_s(Wcol + o, (size_t)out, x, in);
}

static float act_apply(int act, float v) {
    if (act == MZ_ACT_RELU) return mz_relu(v);
    if (act == MZ_ACT_TANH) return det_tanhf(v);
    return v;
}

/* Flux BatchNorm in test mode: λ.(γ .* (x .- μ) ./ sqrt.(σ² .+ ϵ) .+ β), μ = 0,
 * σ² = 1, ϵ = 1f-5 (the running statistics the reference never updates) */
static float bn_apply(const OLayer* l, const float* P, int o, float t) {
    const float s = sqrtf(1.0f + 1e-5f);
    const float xh = (t - 0.0f) / s;
    return P[l->bnoff + l->out + o] * xh + P[l->bnoff + o];
}

/* Flux Dense: σ.(W*x .+ b); make_dense with use_batch_norm (Learning.jl:70-78):
 * Dense(in, out) then BatchNorm(out, relu) in test mode (bn_apply) */
static void dense_fwd(const OLayer* l, const float* P, const float* x, float* y) {
    for (int o = 0; o < l->out; ++o) {
        float t = mz_dot(P + l->woff, l->out, l->in, o, x) + P[l->boff + o];
        if (l->bn) t = bn_apply(l, P, o, t);
        y[o] = act_apply(l->act, t);
    }
}

/* Flux Conv (zero padding, kernel flipped) on a (Wi, Hi, cin) column-major
 * activation: the im2col row of output position (w, h) is, for k = i +
 * kw*j + kw*kh*c (the weight's column-major order), x[sw*w + (kw-1-i) - pw,
 * sh*h + (kh-1-j) - ph, c] (0 outside the board).  Then bias, BatchNorm, the
 * saved block input, act. */
static void conv_fwd(const OLayer* l, const float* P, const float* x, float* y, const float* res) {
    const int W = l->W, H = l->H, Pn = W * H, K = l->kw * l->kh * l->in;
    const int Wi = l->Wi, Hi = l->Hi, Pi = Wi * Hi;
    float* col = (float*)malloc(sizeof(float) * (size_t)K);
    for (int hh = 0; hh < H; ++hh)
        for (int ww = 0; ww < W; ++ww) {
            for (int c = 0; c < l->in; ++c)
                for (int j = 0; j < l->kh; ++j)
                    for (int i = 0; i < l->kw; ++i) {
                        const int sx = l->sw * ww + (l->kw - 1 - i) - l->pw;
                        const int sy = l->sh * hh + (l->kh - 1 - j) - l->ph;
                        const int k = i + l->kw * j + l->kw * l->kh * c;
                        col[k] = (sx >= 0 && sx < Wi && sy >= 0 && sy < Hi) ? x[sx + Wi * sy + Pi * c] : 0.0f;
                    }
            const int p = ww + W * hh;
            for (int o = 0; o < l->out; ++o) {
                float t = mz_dot_s(P + l->woff + (size_t)K * o, 1, col, K) + P[l->boff + o];
                if (l->bn) t = bn_apply(l, P, o, t);
                if (l->res_add) t = t + res[p + (size_t)Pn * o];
                y[p + (size_t)Pn * o] = act_apply(l->act, t);
            }
        }
    free(col);
}

/* NNlib meanpool (0.7): the in-board window entries summed in f32, rows of
 * the window (j) outer and columns (i) inner, times Float32(1/prod(k)) —
 * padded entries count in the divisor (the window is never flipped). */
static void pool_fwd(const OLayer* l, const float* x, float* y) {
    const int W = l->W, H = l->H, Wi = l->Wi, Hi = l->Hi;
    const float inv = 1.0f / (float)(l->kw * l->kh);
    for (int c = 0; c < l->in; ++c)
        for (int hh = 0; hh < H; ++hh)
            for (int ww = 0; ww < W; ++ww) {
                float m = 0.0f;
                for (int j = 0; j < l->kh; ++j)
                    for (int i = 0; i < l->kw; ++i) {
                        const int sx = l->sw * ww + i - l->pw, sy = l->sh * hh + j - l->ph;
                        if (sx >= 0 && sx < Wi && sy >= 0 && sy < Hi) m = m + x[sx + Wi * sy + Wi * Hi * c];
                    }
                y[ww + W * hh + W * H * c] = inv * m;
            }
}

/* NNlib softmax over n entries: max, exp(x - max), sequential sum, divide. */
static void softmax_n(const float* x, int n, float* y) {
    float m = x[0];
    for (int i = 1; i < n; ++i) m = m > x[i] ? m : x[i];
    float s = 0.0f;
    for (int i = 0; i < n; ++i) { y[i] = det_expf(x[i] - m); s = s + y[i]; }
    for (int i = 0; i < n; ++i) y[i] = y[i] / s;
}

static void run_chain(const ONet* net, int part, const float* P, const float* x, float* y) {
    const size_t sz = (size_t)net->maxact;
    float* a = (float*)malloc(sizeof(float) * sz * 3);
    float *b = a + sz, *res = a + 2 * sz;
    const float* cur = x;
    for (int i = 0; i < net->n[part]; ++i) {
        const OLayer* l = &net->L[part][i];
        float* dst = (i & 1) ? b : a;
        if (l->res_save) memcpy(res, cur, sizeof(float) * (size_t)olayer_insize(l));
        if (l->pool) pool_fwd(l, cur, dst);
        else if (l->conv) conv_fwd(l, P, cur, dst, res);
        else dense_fwd(l, P, cur, dst);
        cur = dst;
    }
    memcpy(y, cur, sizeof(float) * (size_t)olayer_outsize(&net->L[part][net->n[part] - 1]));
    free(a);
}

/* forward of one sample; REPR: out0 = h; PRED: out0 = value, out1 = policy;
 * DYN: out0 = h', out1 = reward.  The Split applies both heads to the trunk
 * output (Learning.jl:68). */
static void net_forward1(const ONet* net, const float* P, const float* x, float* out0, float* out1) {
    float* t = (float*)malloc(sizeof(float) * (size_t)net->maxact);
    run_chain(net, 0, P, x, net->n[1] ? t : out0);
    if (net->n[1]) {
        run_chain(net, 1, P, t, out0);
        if (net->softmax_head2) {
            float lg[MAXA];
            run_chain(net, 2, P, t, lg);
            softmax_n(lg, net->L[2][net->n[2] - 1].out, out1);
        } else {
            run_chain(net, 2, P, t, out1);
        }
    }
    free(t);
}

EXPORT int ora_hidden_size(const mz_config* c, const ora_nethp* hp) { return nethp_hidden(c, hp); }

EXPORT size_t ora_param_count(const mz_config* c, const ora_nethp* hp, int which) {
    ONet n; onet_build(&n, which, c, hp); return n.nparams;
}

/* batched forward, column-major (features, n) */
EXPORT void ora_net_forward(const mz_config* c, const ora_nethp* hp, int which, const float* P,
                            const float* x, int n, float* out0, float* out1) {
    ONet net; onet_build(&net, which, c, hp);
    int in = olayer_insize(&net.L[0][0]);
    int o0 = which == MZ_NET_PRED ? 1 : nethp_hidden(c, hp);
    int o1 = which == MZ_NET_PRED ? c->action_space_size : 1;
    for (int i = 0; i < n; ++i)
        net_forward1(&net, P, x + (size_t)i * in, out0 + (size_t)i * o0, out1 ? out1 + (size_t)i * o1 : NULL);
}

/* ===================================================================== MCTS
 * SelfPlay.jl:22-306 */
typedef struct {
    int visit_count;      /* :63 */
    int to_play;          /* :64 default 1 */
    float prior;          /* :65 */
    float value_sum;      /* :66 */
    int expanded;         /* children !== nothing (:72) */
    int child[MAXA];      /* node index per action (0-based action), -1 = none */
    int hslot;            /* hidden_state (expanded slot), -1 = nothing */
    float reward;         /* :69 */
    int eslot;            /* expanded-node slot (0 = root, s+1 = sim s), -1 */
} ONode;

typedef struct { float min, max; } MinMax;                       /* :22-25 */
static void mm_update(MinMax* m, float v) {                       /* :27-31 */
    m->min = m->min < v ? m->min : v;
    m->max = m->max > v ? m->max : v;
}
static float mm_normalize(const MinMax* m, float v) {             /* :33-39 */
    if (m->max > m->min) return (v - m->min) / (m->max - m->min);
    return v;
}

typedef struct {
    const mz_config* c;
    const ora_nethp* hp;
    ONet nrep, npred, ndyn;
    const float *Prep, *Ppred, *Pdyn;
    uint64_t seed;
    int H, A, S;
    ONode* nodes; int nn;
    float* hid;            /* (S+1) * H */
} OCtx;

static float node_value(const ONode* n) {                         /* :76-82 */
    if (n->visit_count == 0) return 0.0f;
    return n->value_sum / (float)n->visit_count;
}

static int new_node(OCtx* X, float prior) {
    ONode* n = &X->nodes[X->nn];
    memset(n, 0, sizeof(*n));
    n->to_play = 1; n->prior = prior; n->hslot = -1; n->eslot = -1;
    for (int a = 0; a < MAXA; ++a) n->child[a] = -1;
    return X->nn++;
}

/* expand_node! (:88-96): priors = softmax over the (already softmaxed, Q3)
 * policy entries of `actions` (the ROOT's legal set at every depth, Q4). */
static void expand_node(OCtx* X, int ni, const uint8_t* legal, int to_play, float reward,
                        const float* policy, int hslot, int eslot) {
    float v[MAXA] = {0}, p[MAXA]; int acts[MAXA], n = 0;
    for (int a = 0; a < X->A; ++a) if (legal[a]) { acts[n] = a; v[n] = policy[a]; ++n; }
    softmax_n(v, n, p);
    for (int i = 0; i < n; ++i) {
        int ci = new_node(X, p[i]);
        X->nodes[ni].child[acts[i]] = ci;
    }
    ONode* node = &X->nodes[ni];
    node->expanded = 1;
    node->to_play = to_play;
    node->reward = reward;
    node->hslot = hslot;
    node->eslot = eslot;
}

/* add_exploration_noise! (:102-109) */
static void add_noise(OCtx* X, int ni, uint32_t game, uint32_t step) {
    ONode* node = &X->nodes[ni];
    int acts[MAXA], n = 0;
    for (int a = 0; a < X->A; ++a) if (node->child[a] >= 0) acts[n++] = a;
    float noise[MAXA];
    mz_dirichlet(X->seed, game, step, n, X->c->dirichlet_alpha, noise);
    float one_m = 1.0f - X->c->exploration_eps;
    for (int i = 0; i < n; ++i) {
        ONode* ch = &X->nodes[node->child[acts[i]]];
        ch->prior = ch->prior * one_m + noise[i] * X->c->exploration_eps;
    }
}

/* ucb_score (:171-184), quirk Q5: pb_c and prior_score in Float64, the sum
 * rounded once to Float32 by the ::Float32 return annotation. */
static float ucb_score(OCtx* X, const ONode* parent, const ONode* child, const MinMax* mm) {
    const mz_config* c = X->c;
    double pb_c = log2((double)(parent->visit_count + c->pb_c_base + 1) / (double)c->pb_c_base)
                  + (double)c->pb_c_init;
    pb_c = pb_c * (sqrt((double)parent->visit_count) / (double)(child->visit_count + 1));
    double prior_score = pb_c * (double)child->prior;
    float value_score = 0.0f;
    if (child->visit_count > 0) {
        float q = node_value(child);
        float t = c->players == 1 ? c->discount * q : c->discount * (-q);
        value_score = mm_normalize(mm, child->reward + t);
    }
    return (float)(prior_score + (double)value_score);
}

/* select_child (:157-166): argmax UCB, uniform tie-break (Philox TIE). */
static int select_child(OCtx* X, int ni, const MinMax* mm, uint32_t game, uint32_t step,
                        int sim, int depth, int* action_out) {
    const ONode* node = &X->nodes[ni];
    float u[MAXA]; int acts[MAXA], n = 0;
    for (int a = 0; a < X->A; ++a) if (node->child[a] >= 0) {
        acts[n] = a; u[n] = ucb_score(X, node, &X->nodes[node->child[a]], mm); ++n;
    }
    float m = u[0];
    for (int i = 1; i < n; ++i) m = m > u[i] ? m : u[i];     /* maximum */
    int ties[MAXA], nt = 0;
    for (int i = 0; i < n; ++i) if (u[i] == m) ties[nt++] = i;
    uint32_t r = mz_rng_u32(X->seed, MZ_RNG_TIE, game, step, ((uint32_t)sim << 12) | (uint32_t)depth);
    int pick = ties[mz_rng_below(r, (uint32_t)nt)];
    *action_out = acts[pick];
    return node->child[acts[pick]];
}

/* backpropagate! (:190-217), quirk Q7 */
static void backpropagate(OCtx* X, const int* path, int len, float value, int to_play, MinMax* mm) {
    const mz_config* c = X->c;
    if (c->players == 1) {
        for (int i = len - 1; i >= 0; --i) {
            ONode* node = &X->nodes[path[i]];
            node->value_sum = node->value_sum + value;
            node->visit_count += 1;
            mm_update(mm, node->reward + c->discount * node_value(node));
            value = node->reward + c->discount * value;
        }
    } else if (c->players == 2) {
        for (int i = len - 1; i >= 0; --i) {
            ONode* node = &X->nodes[path[i]];
            if (node->to_play == to_play) node->value_sum = node->value_sum + value;
            else node->value_sum = node->value_sum - value;
            node->visit_count += 1;
            mm_update(mm, node->reward + c->discount * node_value(node));
            if (node->to_play == to_play) value = -node->reward;
            else value = node->reward + c->discount * value;
        }
    }
    /* > 2 players: the reference builds an ErrorException it never throws (:214) */
}

/* run_mcts (:230-285).  Returns the root node index.  `sims` statistics:
 * stats[0] += sum of select depths, stats[1] = max depth. */
static int run_mcts(OCtx* X, const float* obs, const uint8_t* legal, int to_play, int exploration,
                    uint32_t game, uint32_t step, int64_t* stats) {
    const mz_config* c = X->c;
    int H = X->H, A = X->A;
    X->nn = 0;
    int root = new_node(X, 0.0f);                                   /* :232 */
    float* h0 = X->hid;                                             /* slot 0 */
    net_forward1(&X->nrep, X->Prep, obs, h0, NULL);                 /* :234 */
    float v0, pol[MAXA];
    net_forward1(&X->npred, X->Ppred, h0, &v0, pol);                /* :239 */
    expand_node(X, root, legal, to_play, 0.0f, pol, 0, 0);          /* :245 */
    if (exploration) add_noise(X, root, game, step);                /* :247-249 */
    MinMax mm = {INFINITY, -INFINITY};                              /* :251 */
    int* path = (int*)malloc(sizeof(int) * (X->S + 2));
    float* sa = (float*)malloc(sizeof(float) * (size_t)olayer_insize(&X->ndyn.L[0][0]));
    for (int it = 0; it < X->S; ++it) {                             /* :254 */
        int node = root, vtp = to_play, len = 0, depth = 0, action = 0;
        path[len++] = node;
        while (X->nodes[node].expanded) {                           /* :261 */
            depth += 1;
            node = select_child(X, node, &mm, game, step, it, depth, &action);
            path[len++] = node;
            vtp = (vtp % c->players) + 1;                           /* mod1(vtp+1, P), :267 */
        }
        if (stats) { stats[0] += depth; if (depth > stats[1]) stats[1] = depth; }
        ONode* parent = &X->nodes[path[len - 2]];                   /* :270 */
        float* ph = X->hid + (size_t)parent->hslot * H;
        float value, pl[MAXA];
        net_forward1(&X->npred, X->Ppred, ph, &value, pl);          /* :271 (Q2) */
        /* make_state_action (:7-14): parent.hidden_state .*= 2 IN PLACE (Q1),
         * action plane Float32(a / |A|) with a 1-based. */
        for (int i = 0; i < H; ++i) ph[i] = ph[i] * 2.0f;
        memcpy(sa, ph, sizeof(float) * H);
        int plane = hid_plane(c, X->hp);
        float aval = (float)((double)(action + 1) / (double)A);
        for (int i = 0; i < plane; ++i) sa[H + i] = aval;
        int slot = it + 1;
        float* nh = X->hid + (size_t)slot * H;
        float reward;
        net_forward1(&X->ndyn, X->Pdyn, sa, nh, &reward);           /* :275 */
        expand_node(X, node, legal, vtp, reward, pl, slot, slot);   /* :280 */
        backpropagate(X, path, len, value, vtp, &mm);               /* :281 */
    }
    free(path);
    free(sa);
    return root;
}

/* select_action (:293-306) with Philox ACTION stream; T==1 samples the
 * integer visit counts exactly. Returns the 0-based action. */
static int select_action(OCtx* X, int root, float temperature, uint32_t game, uint32_t step) {
    const ONode* node = &X->nodes[root];
    int acts[MAXA], cnt[MAXA], n = 0;
    for (int a = 0; a < X->A; ++a) if (node->child[a] >= 0) {
        acts[n] = a; cnt[n] = X->nodes[node->child[a]].visit_count; ++n;
    }
    uint32_t r = mz_rng_u32(X->seed, MZ_RNG_ACTION, game, step, 0);
    if (temperature == 0.0f) {
        int best = 0;
        for (int i = 1; i < n; ++i) if (cnt[i] > cnt[best]) best = i;
        return acts[best];
    }
    if (isinf(temperature)) return acts[mz_rng_below(r, (uint32_t)n)];
    if (temperature == 1.0f) {
        uint32_t tot = 0;
        for (int i = 0; i < n; ++i) tot += (uint32_t)cnt[i];
        if (tot == 0) return acts[mz_rng_below(r, (uint32_t)n)];
        uint32_t t = mz_rng_below(r, tot), cum = 0;
        for (int i = 0; i < n; ++i) { cum += (uint32_t)cnt[i]; if (cum > t) return acts[i]; }
        return acts[n - 1];
    }
    float e = 1.0f / temperature;
    float w[MAXA], s = 0.0f;
    for (int i = 0; i < n; ++i) {
        w[i] = cnt[i] > 0 ? (float)det_exp(det_log((double)cnt[i]) * (double)e) : 0.0f;
        s = s + w[i];
    }
    float u = (float)(r >> 8) * 5.9604644775390625e-08f * s;
    float cum = 0.0f;
    for (int i = 0; i < n; ++i) { cum = cum + w[i]; if (cum > u) return acts[i]; }
    return acts[n - 1];
}

static void ctx_init(OCtx* X, const mz_config* c, const ora_nethp* hp, const float* Prep,
                     const float* Ppred, const float* Pdyn, uint64_t seed) {
    X->c = c; X->hp = hp;
    onet_build(&X->nrep, MZ_NET_REPR, c, hp);
    onet_build(&X->npred, MZ_NET_PRED, c, hp);
    onet_build(&X->ndyn, MZ_NET_DYN, c, hp);
    X->Prep = Prep; X->Ppred = Ppred; X->Pdyn = Pdyn;
    X->seed = seed;
    X->H = nethp_hidden(c, hp); X->A = c->action_space_size; X->S = c->num_iters;
    X->nodes = (ONode*)malloc(sizeof(ONode) * (size_t)(1 + (X->S + 1) * X->A));
    X->hid = (float*)malloc(sizeof(float) * (size_t)(X->S + 1) * X->H);
}
static void ctx_free(OCtx* X) { free(X->nodes); free(X->hid); }

/* store_search_stats! (:115-122) for one game */
static void search_stats(OCtx* X, int root, float* child_visits, float* root_value) {
    const ONode* node = &X->nodes[root];
    int sum = 0;
    for (int a = 0; a < X->A; ++a) if (node->child[a] >= 0) sum += X->nodes[node->child[a]].visit_count;
    for (int a = 0; a < X->A; ++a)
        child_visits[a] = node->child[a] >= 0
            ? (float)((double)X->nodes[node->child[a]].visit_count / (double)sum) : 0.0f;
    *root_value = node_value(node);
}

/* Dump the tree in the engine's slot layout (see mz_debug_tree). */
static void dump_tree(OCtx* X, int g, int G, int32_t* eN, float* eW, float* eP, float* eR,
                      int32_t* ech, int32_t* ntp) {
    int S = X->S, A = X->A;
    for (int i = 0; i < X->nn; ++i) {
        const ONode* n = &X->nodes[i];
        if (!n->expanded) continue;
        int e = n->eslot;
        if (ntp) ntp[(size_t)g * (S + 1) + e] = n->to_play;
        for (int a = 0; a < A; ++a) {
            size_t k = ((size_t)g * (S + 1) + e) * A + a;
            int ci = n->child[a];
            const ONode* ch = ci >= 0 ? &X->nodes[ci] : NULL;
            if (eN) eN[k] = ch ? ch->visit_count : 0;
            if (eW) eW[k] = ch ? ch->value_sum : 0.0f;
            if (eP) eP[k] = ch ? ch->prior : 0.0f;
            if (eR) eR[k] = ch && ch->expanded ? ch->reward : 0.0f;
            if (ech) ech[k] = ch && ch->expanded ? ch->eslot : -1;
        }
    }
    (void)G;
}

/* Batched search: the ABI of mz_mcts_search, on the CPU. */
EXPORT int ora_mcts_search(const mz_config* c, const ora_nethp* hp, const float* Prep, const float* Ppred,
                           const float* Pdyn, uint64_t seed, int G, const float* obs,
                           const uint8_t* legal_mask, const int32_t* to_play, int exploration,
                           uint32_t rng_step, uint32_t game_offset, float temperature,
                           float* child_visits, float* root_value, int32_t* action_out,
                           int32_t* eN, float* eW, float* eP, float* eR, int32_t* ech, int32_t* ntp,
                           int64_t* stats) {
    OCtx X; ctx_init(&X, c, hp, Prep, Ppred, Pdyn, seed);
    int A = X.A;
    int in = olayer_insize(&X.nrep.L[0][0]);
    for (int g = 0; g < G; ++g) {
        uint32_t gid = game_offset + (uint32_t)g;
        int root = run_mcts(&X, obs + (size_t)g * in, legal_mask + (size_t)g * A, to_play[g],
                            exploration, gid, rng_step, stats);
        search_stats(&X, root, child_visits + (size_t)g * A, root_value + g);
        action_out[g] = select_action(&X, root, temperature, gid, rng_step) + 1;
        if (eN || eW || eP || eR || ech || ntp) dump_tree(&X, g, G, eN, eW, eP, eR, ech, ntp);
    }
    ctx_free(&X);
    return 0;
}

/* ============================================================== TicTacToe
 * games/tictactoe/game.jl, quirk Q14.  Board = BitArray(3,3,3) planes
 * [p1, p2, empty]; action a -> CartesianIndices((3,3))[a] = cell a-1.    */
typedef struct { uint8_t b[27]; int player; } OTTT;

static const int LINES[8][3] = {{0,3,6},{1,4,7},{2,5,8},{0,1,2},{3,4,5},{6,7,8},{0,4,8},{6,4,2}};

static void ttt_reset(OTTT* e) {                                   /* :15-20 */
    memset(e->b, 0, 27); for (int i = 0; i < 9; ++i) e->b[18 + i] = 1; e->player = 1;
}
/* is_win(env, _): checks env.player's plane (the player TO MOVE), :102-115 */
static int ttt_is_win(const OTTT* e) {
    const uint8_t* pl = e->b + 9 * (e->player - 1);
    for (int l = 0; l < 8; ++l) if (pl[LINES[l][0]] && pl[LINES[l][1]] && pl[LINES[l][2]]) return 1;
    return 0;
}
static void ttt_legal(const OTTT* e, uint8_t* mask) {               /* :35-43 */
    int w = ttt_is_win(e);
    for (int i = 0; i < 9; ++i) mask[i] = w ? 0 : e->b[18 + i];
}
static void ttt_step(OTTT* e, int a1) {                             /* :45-52 */
    int c = a1 - 1;
    e->b[18 + c] = 0; e->b[9 * (e->player - 1) + c] = 1;
    e->player = (e->player % 2) + 1;
}
/* state-table entry built by walk (:117-147): winner = 1 if the side to
 * move has a line (labelled 1 whoever owns it), terminated = full || win. */
static int ttt_terminated(const OTTT* e) {
    int empty = 0; for (int i = 0; i < 9; ++i) empty |= e->b[18 + i];
    return !(empty && !ttt_is_win(e));
}
static float ttt_reward(const OTTT* e, int p) {                     /* :87-100 */
    if (!ttt_terminated(e)) return 0.0f;
    if (!ttt_is_win(e)) return 0.0f;
    return p == 1 ? 1.0f : -1.0f;
}

EXPORT void ora_ttt_step(uint8_t* board, int32_t* player, int action, uint8_t* legal_out,
                         float* reward_out, int32_t* done_out) {
    OTTT e; memcpy(e.b, board, 27); e.player = *player;
    int p = e.player;
    ttt_step(&e, action);
    memcpy(board, e.b, 27); *player = e.player;
    if (legal_out) ttt_legal(&e, legal_out);
    if (reward_out) *reward_out = ttt_reward(&e, p);
    if (done_out) *done_out = ttt_terminated(&e);
}

/* get_stacked_observations (SelfPlay.jl:128-149), Q15: channels
 * [obs_t, action plane (raw action id), obs_{t-1}, ...], zeros before t=1.
 * obs_hist is (W*H*C, T) column-major; index is 1-based. */
EXPORT void ora_stacked_obs(const mz_config* c, const float* obs_hist, const int32_t* action_hist,
                            int index, float* out) {
    int plane = c->observation_shape[0] * c->observation_shape[1];
    int osz = plane * c->observation_shape[2];
    memcpy(out, obs_hist + (size_t)(index - 1) * osz, sizeof(float) * osz);
    float* o = out + osz;
    for (int past = index - 1; past >= index - c->stacked_observations; --past) {
        if (past >= 1) {
            for (int i = 0; i < plane; ++i) o[i] = (float)action_hist[past - 1];
            memcpy(o + plane, obs_hist + (size_t)(past - 1) * osz, sizeof(float) * osz);
        } else {
            memset(o, 0, sizeof(float) * (plane + osz));
        }
        o += plane + osz;
    }
}

/* play_game (SelfPlay.jl:330-382) for one TicTacToe game, opponent "self".
 * Move t uses RNG step step0 + t.  Outputs are GameHistory columns sized
 * for max_moves+1 moves; returns the number of moves T.                   */
EXPORT int ora_play_game(const mz_config* c, const ora_nethp* hp, const float* Prep, const float* Ppred,
                         const float* Pdyn, uint64_t seed, uint32_t game_id, uint32_t step0,
                         float temperature, float* obs_hist, int32_t* action_hist, float* reward_hist,
                         int32_t* to_play_hist, float* child_visits, float* root_values) {
    OCtx X; ctx_init(&X, c, hp, Prep, Ppred, Pdyn, seed);
    OTTT env; ttt_reset(&env);
    int A = X.A, T = 0, done = 0;
    float stacked[1024];
    while (!done && T <= c->max_moves) {                           /* :343 */
        float temp = temperature;
        if (c->temperature_threshold >= 0 && T >= c->temperature_threshold) temp = 0.0f;
        int p = env.player;                                         /* :351 */
        for (int i = 0; i < 27; ++i) obs_hist[(size_t)T * 27 + i] = (float)env.b[i];   /* :352 */
        ora_stacked_obs(c, obs_hist, action_hist, T + 1, stacked);  /* :355 */
        uint8_t legal[MAXA]; ttt_legal(&env, legal);
        uint32_t step = step0 + (uint32_t)T;
        int root = run_mcts(&X, stacked, legal, p, 1, game_id, step, NULL);   /* :359 */
        int a = select_action(&X, root, temp, game_id, step) + 1; /* :360 */
        ttt_step(&env, a);                                          /* :366 */
        float r = ttt_reward(&env, p);                              /* :367 */
        done = ttt_terminated(&env);                                /* :368 */
        search_stats(&X, root, child_visits + (size_t)T * A, root_values + T);   /* :375 */
        action_hist[T] = a; reward_hist[T] = r; to_play_hist[T] = p; /* :377-379 */
        ++T;
    }
    ctx_free(&X);
    return T;
}

/* ========================================================= replay buffer
 * src/ReplayBuffer.jl.  A history is passed as column arrays of length T. */
typedef struct {
    int32_t T;
    const float* obs;          /* (27, T) observation_history */
    const int32_t* actions;    /* (T) action_history, 1-based ids */
    const float* rewards;      /* (T) reward_history */
    const int32_t* to_play;    /* (T) to_play_history */
    const float* child_visits; /* (A, T) */
    const float* root_values;  /* (T) */
} OHist;

/* discount^n: Julia's Float32^Int (llvm.pow.f32) ≈ round-to-f32 of pow(f64) */
static float disc_pow(float g, int n) { return (float)pow((double)g, (double)n); }

/* compute_target_value (:5-20), Q9; index is 1-based */
EXPORT float ora_compute_target_value(const mz_config* c, const OHist* h, int index) {
    int bi = index + c->td_steps;
    float value;
    if (bi < h->T) {
        float rv = h->root_values[bi - 1];
        float last = h->to_play[bi - 1] == h->to_play[index - 1] ? rv : -rv;
        value = last * disc_pow(c->discount, c->td_steps);
        for (int i = 1; i <= c->td_steps + 1; ++i) {                 /* enumerate(reward_history[index:bi]) */
            float r = h->rewards[index + i - 2];
            float sr = h->to_play[index - 1] == h->to_play[index + i - 1] ? r : -r;
            value = value + sr * disc_pow(c->discount, i);
        }
    } else {
        value = 0.0f;
    }
    return value;
}

/* make_target (:25-50); absorbing-state actions from Philox ABSORB */
static void make_target(const mz_config* c, const OHist* h, int state_index, uint64_t seed,
                        uint32_t sample, uint32_t step, float* tv, float* tr, float* tp, float* ta) {
    int A = c->action_space_size, K = c->num_unroll_steps;
    for (int k = 0; k <= K; ++k) {
        int ci = state_index + k;
        if (ci < h->T) {
            tv[k] = ora_compute_target_value(c, h, ci);
            tr[k] = h->rewards[ci - 1];
            for (int a = 0; a < A; ++a) tp[(size_t)k * A + a] = h->child_visits[(size_t)(ci - 1) * A + a];
            ta[k] = (float)h->actions[ci - 1];
        } else if (ci == h->T) {
            tv[k] = 0.0f;
            tr[k] = h->rewards[ci - 1];
            for (int a = 0; a < A; ++a) tp[(size_t)k * A + a] = 1.0f / (float)A;
            ta[k] = (float)h->actions[ci - 1];
        } else {
            tv[k] = 0.0f; tr[k] = 0.0f;
            for (int a = 0; a < A; ++a) tp[(size_t)k * A + a] = 1.0f / (float)A;
            ta[k] = (float)(mz_rng_below(mz_rng_u32(seed, MZ_RNG_ABSORB, sample, step, (uint32_t)k), (uint32_t)A) + 1);
        }
    }
}

/* get_batch (:188-217) over a buffer of n histories (ids first_id..).
 * Uniform sampling (PER=false): sample_n_games (:102), sample_position (:80).
 * Outputs column-major as the reference's batch tuple; idx_out (2,B) =
 * (game_id, position). */
EXPORT void ora_get_batch(const mz_config* c, const OHist* hist, int n, int first_id, uint64_t seed,
                          uint32_t step, float* obs, float* actions, float* values, float* rewards,
                          float* policies, float* gscale, int32_t* idx_out) {
    int A = c->action_space_size, K = c->num_unroll_steps, B = c->batch_size;
    int osz = c->observation_shape[0] * c->observation_shape[1] *
              (c->observation_shape[2] * (c->stacked_observations + 1) + c->stacked_observations);
    for (int b = 0; b < B; ++b) {
        int gi = (int)mz_rng_below(mz_rng_u32(seed, MZ_RNG_GAME, (uint32_t)b, step, 0), (uint32_t)n);
        const OHist* h = &hist[gi];
        int pos = (int)mz_rng_below(mz_rng_u32(seed, MZ_RNG_POS, (uint32_t)b, step, 0), (uint32_t)h->T) + 1;
        make_target(c, h, pos, seed, (uint32_t)b, step, values + (size_t)b * (K + 1),
                    rewards + (size_t)b * (K + 1), policies + (size_t)b * (K + 1) * A,
                    actions + (size_t)b * (K + 1));
        ora_stacked_obs(c, h->obs, h->actions, pos, obs + (size_t)b * osz);
        int gs = h->T + 1 - pos;                                     /* :212 */
        gscale[b] = (float)(K < gs ? K : gs);
        idx_out[2 * b] = first_id + gi; idx_out[2 * b + 1] = pos;
    }
}

/* ================================================================ learner
 * Learning.jl:261-413 in ref_semantics (Q10, Q11). */

/* logsoftmax (NNlib) + logitcrossentropy for one (A) column */
static float policy_ce(const float* yhat, const float* y, int A) {
    float m = yhat[0];
    for (int i = 1; i < A; ++i) m = m > yhat[i] ? m : yhat[i];
    float s = 0.0f;
    for (int i = 0; i < A; ++i) s = s + det_expf(yhat[i] - m);
    float ls = det_logf(s);
    float ce = 0.0f;
    for (int i = 0; i < A; ++i) ce = ce + y[i] * ((yhat[i] - m) - ls);
    return -ce;
}

/* The forward unroll: predictions values (K+1,B), policies (A,K+1,B),
 * rewards (K+1,B) exactly as Learning.jl:347-370 builds them (Q10). */
EXPORT void ora_unroll(const mz_config* c, const ora_nethp* hp, const float* Prep, const float* Ppred,
                       const float* Pdyn, int B, const float* obs, const float* actions,
                       float* pv, float* pp, float* pr) {
    ONet nr, np, nd;
    onet_build(&nr, MZ_NET_REPR, c, hp); onet_build(&np, MZ_NET_PRED, c, hp); onet_build(&nd, MZ_NET_DYN, c, hp);
    int H = nethp_hidden(c, hp), A = c->action_space_size, K = c->num_unroll_steps;
    int in = olayer_insize(&nr.L[0][0]);
    int plane = hid_plane(c, hp);
    float* h = (float*)malloc(sizeof(float) * (size_t)H);
    float* sa = (float*)malloc(sizeof(float) * (size_t)(H + plane));
    float v, pol[MAXA];
    for (int b = 0; b < B; ++b) {
        net_forward1(&nr, Prep, obs + (size_t)b * in, h, NULL);          /* :347 */
        net_forward1(&np, Ppred, h, &v, pol);                            /* :351 */
        pv[(size_t)b * (K + 1)] = v; pr[(size_t)b * (K + 1)] = 0.0f;      /* :352 zeros */
        memcpy(pp + (size_t)b * (K + 1) * A, pol, sizeof(float) * A);
        for (int i = 1; i <= K; ++i) {                                   /* :355 */
            net_forward1(&np, Ppred, h, &v, pol);                        /* :356 */
            /* make_dynamics_input (:293-304): actions ./= |A| (Float32), 2h */
            float a = actions[(size_t)b * (K + 1) + (i - 1)] / (float)A;
            for (int j = 0; j < H; ++j) sa[j] = h[j] * 2.0f;
            for (int j = 0; j < plane; ++j) sa[H + j] = a;
            float r;
            net_forward1(&nd, Pdyn, sa, h, &r);                          /* :362 */
            pv[(size_t)b * (K + 1) + i] = v;                             /* :367-369 */
            pr[(size_t)b * (K + 1) + i] = r;
            memcpy(pp + ((size_t)b * (K + 1) + i) * A, pol, sizeof(float) * A);
        }
    }
    free(h); free(sa);
}

/* loss (:261-288) data terms.  Julia's Float32 `sum`/`mean` are pairwise and
 * not reproducible offline; the restatement fixes one order, the
 * engine's lg_fold (muzero.jl_amd/csrc/mz_learner_device.h): each sample's
 * K+1 step terms in ascending k in f32, then the cross-sample sums in f64 —
 * 64 lanes (sample j on lane j mod 64, ascending j), folded by the xor
 * butterfly (offsets 32..1) into lane 0.  Both sides therefore round once
 * from a near-exact f64 sum.                                                 */
static double fold64(const double* lanes) {
    double x[64], y[64];
    memcpy(x, lanes, sizeof(x));
    for (int o = 32; o >= 1; o >>= 1) {
        for (int l = 0; l < 64; ++l) y[l] = x[l] + x[l ^ o];
        memcpy(x, y, sizeof(x));
    }
    return x[0];
}

EXPORT void ora_losses_w(const mz_config* c, int B, const float* pv, const float* pp, const float* tv,
                         const float* tp, const float* gscale, const float* wts, float* value_loss,
                         float* policy_loss) {
    int A = c->action_space_size, K = c->num_unroll_steps;
    double sv[64] = {0}, sc[64] = {0}, sg[64] = {0};
    for (int j = 0; j < B; ++j) {
        float s = 0.0f, ce = 0.0f;
        for (int k = 0; k <= K; ++k) {
            float d = pv[(size_t)j * (K + 1) + k] - tv[(size_t)j * (K + 1) + k];
            s = s + d * d;                                           /* mse, :273 */
            ce = ce + policy_ce(pp + ((size_t)j * (K + 1) + k) * A, tp + ((size_t)j * (K + 1) + k) * A, A);
        }
        float w = wts ? wts[j] : 1.0f;                               /* PER weight_batch, :271-285 */
        sv[j & 63] += (double)((s / gscale[j]) * w);
        sc[j & 63] += (double)ce;                                    /* Σ_k CE_k */
        sg[j & 63] += (double)w / (double)gscale[j];
    }
    /* value: mean((sum(x, dims=1) ./ g) .* w) */
    *value_loss = (float)(fold64(sv) / (double)B);
    /* policy: (1,1,B) ./ (1,B) broadcast to (1,B,B) then mean (Q11):
     * Σ_j CE_j · Σ_i w_i/g_i / B² */
    *policy_loss = (float)(fold64(sc) * fold64(sg) / ((double)B * (double)B));
}

EXPORT void ora_losses(const mz_config* c, int B, const float* pv, const float* pp, const float* tv,
                       const float* tp, const float* gscale, float* value_loss, float* policy_loss) {
    ora_losses_w(c, B, pv, pp, tv, tp, gscale, NULL, value_loss, policy_loss);
}

/* sum(sqnorm, params) (:287) in f64, in the engine's fixed order
 * (lg_l2_slice + lg_tree256 + lg_fold): 128 slices of 256 threads (MZ_L2_BLOCKS),
 * thread t of slice b summing elements b·256 + t + j·32768 in ascending j, a
 * pairwise tree over the 256 threads (offsets 128..1), then lane l of the
 * 64-lane butterfly holding slices l and l + 64 (summed in that order).      */
EXPORT double ora_sqnorm(const float* P, size_t n) {
    enum { NB = 128, NT = 256 };
    const size_t stride = (size_t)NB * NT;
    double part[NB], lanes[64];
    for (int b = 0; b < NB; ++b) {
        double red[NT];
        for (int t = 0; t < NT; ++t) {
            double s = 0.0;
            for (size_t i = (size_t)b * NT + t; i < n; i += stride) s += (double)P[i] * (double)P[i];
            red[t] = s;
        }
        for (int o = NT / 2; o > 0; o >>= 1)
            for (int t = 0; t < o; ++t) red[t] += red[t + o];
        part[b] = red[0];
    }
    for (int l = 0; l < 64; ++l) {
        double s = 0.0;
        for (int b = l; b < NB; b += 64) s += part[b];
        lanes[l] = s;
    }
    return fold64(lanes);
}

/* Flux 0.12 ADAMW() = Optimiser(ADAM(η, (0.9, 0.999)), WeightDecay(0));
 * apply!(ADAM): mt, vt in Float32 arrays, arithmetic in Float64 (β, η are
 * Float64), Δ^2 in Float32 (literal_pow); WeightDecay(0) is the identity.
 * The gradient is 2θ (Q11).  bp = βp state (Float64[β1^t, β2^t]).        */
EXPORT void ora_adam_2theta(float* P, float* m, float* v, size_t n, const double* bp, double eta) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    for (size_t i = 0; i < n; ++i) {
        float g = P[i] * 2.0f;
        m[i] = (float)(b1 * (double)m[i] + (1.0 - b1) * (double)g);
        float g2 = g * g;
        v[i] = (float)(b2 * (double)v[i] + (1.0 - b2) * (double)g2);
        float d = (float)((double)m[i] / (1.0 - bp[0]) / (sqrt((double)v[i] / (1.0 - bp[1])) + eps) * eta);
        P[i] = P[i] - d;
    }
}

/* The same update with an explicit gradient g (the data-parallel step:
 * g = (Σ_ranks data term)·(1/world) + 2θ).                      */
EXPORT void ora_adam_grad(float* P, float* m, float* v, const float* gr, size_t n, const double* bp, double eta) {
    const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
    for (size_t i = 0; i < n; ++i) {
        float g = gr[i];
        m[i] = (float)(b1 * (double)m[i] + (1.0 - b1) * (double)g);
        float g2 = g * g;
        v[i] = (float)(b2 * (double)v[i] + (1.0 - b2) * (double)g2);
        float d = (float)((double)m[i] / (1.0 - bp[0]) / (sqrt((double)v[i] / (1.0 - bp[1])) + eps) * eta);
        P[i] = P[i] - d;
    }
}

/* ParameterSchedulers 0.2.3 Cos(λ0, λ1, period) with Stateful (1-based t):
 * |λ0−λ1|·(1 + cos(2π(t−1)/period))/2 + min(λ0, λ1). */
EXPORT double ora_cos_schedule(double l0, double l1, int period, int t) {
    double range = fabs(l0 - l1), off = l0 < l1 ? l0 : l1;
    double a = 6.283185307179586 * (double)(t - 1) / (double)period;
    return range * (1.0 + cos(a)) / 2.0 + off;
}

/* One full ref_semantics learner step: forward unroll + losses + ADAM on
 * all three nets; bp is advanced (βp .= βp .* β).                          */
/* ... with PER importance weights wts (B) or NULL (Learning.jl:271-285) */
EXPORT void ora_learner_step_w(const mz_config* c, const ora_nethp* hp, float* Prep, float* Ppred, float* Pdyn,
                               float* m_all, float* v_all, double* bp, int B, const float* obs,
                               const float* actions, const float* tv, const float* tp, const float* gscale,
                               const float* wts, double eta, float* losses) {
    int A = c->action_space_size, K = c->num_unroll_steps;
    float* pv = (float*)malloc(sizeof(float) * (size_t)B * (K + 1));
    float* pr = (float*)malloc(sizeof(float) * (size_t)B * (K + 1));
    float* pp = (float*)malloc(sizeof(float) * (size_t)B * (K + 1) * A);
    ora_unroll(c, hp, Prep, Ppred, Pdyn, B, obs, actions, pv, pp, pr);
    ora_losses_w(c, B, pv, pp, tv, tp, gscale, wts, &losses[0], &losses[2]);
    losses[1] = 0.0f;                                  /* intermediate_rewards = false */
    size_t n0 = ora_param_count(c, hp, MZ_NET_REPR), n1 = ora_param_count(c, hp, MZ_NET_PRED),
           n2 = ora_param_count(c, hp, MZ_NET_DYN);
    losses[3] = (float)ora_sqnorm(Prep, n0);
    losses[4] = (float)ora_sqnorm(Ppred, n1);
    losses[5] = (float)ora_sqnorm(Pdyn, n2);
    ora_adam_2theta(Prep, m_all, v_all, n0, bp, eta);
    ora_adam_2theta(Ppred, m_all + n0, v_all + n0, n1, bp, eta);
    ora_adam_2theta(Pdyn, m_all + n0 + n1, v_all + n0 + n1, n2, bp, eta);
    bp[0] = bp[0] * 0.9; bp[1] = bp[1] * 0.999;
    free(pv); free(pr); free(pp);
}
EXPORT void ora_learner_step(const mz_config* c, const ora_nethp* hp, float* Prep, float* Ppred, float* Pdyn,
                             float* m_all, float* v_all, double* bp, int B, const float* obs,
                             const float* actions, const float* tv, const float* tp, const float* gscale,
                             double eta, float* losses) {
    ora_learner_step_w(c, hp, Prep, Ppred, Pdyn, m_all, v_all, bp, B, obs, actions, tv, tp, gscale, NULL, eta,
                       losses);
}

/* ==================================================================== PER
 * Prioritized replay (conf.PER; ReplayBuffer.jl:73-107, 133-145, 168-183,
 * 188-217; Learning.jl:261-288, 400-404).  The reference's PER path cannot
 * run (update_priorities! calls minimum(a, b) and assigns a K+2-element slice
 * from K+1 priorities); this restates its intended reading.  Julia's
 * rand(rng, Categorical(p)) draws from MersenneTwister (not reproducible
 * offline): the restatement draws u from the Philox GAME / POS streams and
 * applies Distributions 0.25's rand(::DiscreteNonParametric) rule — the first
 * index whose ascending running sum of p exceeds u (advance while cp <= u).  */

/* |x|^alpha as Julia's Float32^Int: f64 repeated multiplication, rounded once */
EXPORT float ora_per_priority(float x, int alpha) {
    double ax = fabs((double)x), r = 1.0;
    for (int i = 0; i < alpha; ++i) r = r * ax;
    return (float)r;
}
/* uniform in [0, 1) from a Philox draw: 24 bits, exact */
static double per_uniform(uint32_t r) { return (double)(r >> 8) * 5.9604644775390625e-08; }
/* Categorical(w ./ sum(w)) (:76, :98): p_i = w_i / S with S the ascending f32
 * sum; the first i whose ascending f32 running sum of p exceeds u (else the
 * last); *prob = p_i */
EXPORT int ora_per_categorical(const float* w, int n, double u, float* prob) {
    float S = 0.0f;
    for (int i = 0; i < n; ++i) S = S + w[i];
    int i = 0;
    float p = w[0] / S, c = p;
    while ((double)c <= u && i < n - 1) { ++i; p = w[i] / S; c = c + p; }
    *prob = p;
    return i;
}
/* save_game's priorities (:136-143): |root_value_i − target_value_i|^alpha,
 * game priority = their max */
EXPORT void ora_per_init(const mz_config* c, const OHist* h, float* prio, float* gprio) {
    float m = 0.0f;
    for (int i = 0; i < h->T; ++i) {
        prio[i] = ora_per_priority(h->root_values[i] - ora_compute_target_value(c, h, i + 1), c->PER_alpha);
        m = i == 0 || prio[i] > m ? prio[i] : m;
    }
    *gprio = m;
}
/* get_batch with PER (:188-217): games by priority (sample_n_games :91-99),
 * positions by priority (sample_position :75-78), importance weights
 * 1/(total_samples · p_game · p_pos) in f32 (:213), normalised by their
 * maximum (:215).  prio is [n][Tmax] (game i = hist[i], oldest first).     */
EXPORT void ora_get_batch_per(const mz_config* c, const OHist* hist, const float* prio, const float* gprio, int n,
                              int Tmax, int first_id, uint64_t seed, uint32_t step, float* obs, float* actions,
                              float* values, float* rewards, float* policies, float* gscale, float* weights,
                              int32_t* idx_out) {
    int A = c->action_space_size, K = c->num_unroll_steps, B = c->batch_size;
    int osz = c->observation_shape[0] * c->observation_shape[1] *
              (c->observation_shape[2] * (c->stacked_observations + 1) + c->stacked_observations);
    long long total = 0;
    for (int i = 0; i < n; ++i) total += hist[i].T;
    float wmax = -INFINITY;
    for (int b = 0; b < B; ++b) {
        float gp, pp;
        int gi = ora_per_categorical(gprio, n, per_uniform(mz_rng_u32(seed, MZ_RNG_GAME, (uint32_t)b, step, 0)), &gp);
        const OHist* h = &hist[gi];
        int pos = ora_per_categorical(prio + (size_t)gi * Tmax, h->T,
                                      per_uniform(mz_rng_u32(seed, MZ_RNG_POS, (uint32_t)b, step, 0)), &pp) + 1;
        weights[b] = 1.0f / ((float)total * gp * pp);
        wmax = weights[b] > wmax ? weights[b] : wmax;
        make_target(c, h, pos, seed, (uint32_t)b, step, values + (size_t)b * (K + 1),
                    rewards + (size_t)b * (K + 1), policies + (size_t)b * (K + 1) * A,
                    actions + (size_t)b * (K + 1));
        ora_stacked_obs(c, h->obs, h->actions, pos, obs + (size_t)b * osz);
        int gs = h->T + 1 - pos;
        gscale[b] = (float)(K < gs ? K : gs);
        idx_out[2 * b] = first_id + gi; idx_out[2 * b + 1] = pos;
    }
    for (int b = 0; b < B; ++b) weights[b] = weights[b] / wmax;
}
/* update_priorities! (:168-183) after a learner step (Learning.jl:400-404):
 * sample i in batch order, if its game is still held, sets positions
 * pos..min(pos+K, len) to |v̂ − v|^alpha of steps 0.., then the game priority
 * to the new maximum (later samples overwrite earlier ones).               */
EXPORT void ora_update_priorities(const mz_config* c, float* prio, float* gprio, const int32_t* lens, int n,
                                  int Tmax, int first_id, int B, const int32_t* idx, const float* pv, const float* tv) {
    int K = c->num_unroll_steps;
    for (int i = 0; i < B; ++i) {
        int gi = idx[2 * i] - first_id, pos = idx[2 * i + 1];
        if (gi < 0 || gi >= n) continue;
        int len = lens[gi], end = pos + K < len ? pos + K : len;
        float* pr = prio + (size_t)gi * Tmax;
        for (int k = pos; k <= end; ++k)
            pr[k - 1] = ora_per_priority(pv[(size_t)i * (K + 1) + (k - pos)] - tv[(size_t)i * (K + 1) + (k - pos)],
                                         c->PER_alpha);
        float m = pr[0];
        for (int k = 1; k < len; ++k) m = pr[k] > m ? pr[k] : m;
        gprio[gi] = m;
    }
}

/* ======================================================= evaluation play
 * competitive_play! (SelfPlay.jl:421-435) = play_game (:330-382) with an
 * opponent at temperature 0, games not saved, for G lockstep slots (the
 * engine's MZ_SP_EVAL mode): the player muzero_player searches (run_mcts +
 * select_action); the other player is "random" — select_opponent_action
 * (:311-325) read as intended (the reference reads `las`, defined only in the
 * "human" branch): a uniform legal action, the rank drawn from the Philox
 * OPPONENT stream keyed (game id, move) — or MuZero too (opponent "self").
 * Each finished game is tallied {games, MuZero wins, opponent wins, draws}:
 * with quirk Q14 a nonzero last reward means the player then to move holds a
 * line (winner = 3 − mover).  TicTacToe only.                               */
EXPORT int ora_eval_play(const mz_config* c, const ora_nethp* hp, const float* Prep, const float* Ppred,
                         const float* Pdyn, uint64_t seed, int G, int moves, uint32_t move0, uint32_t game_offset,
                         int random_opponent, int muzero_player, float temperature, int64_t* tally,
                         int32_t* slot_len, uint8_t* slot_board, int32_t* slot_player) {
    const int A = c->action_space_size, Tm = c->max_moves + 1, OS = 27;
    if (A != 9) return -1;
    OCtx X; ctx_init(&X, c, hp, Prep, Ppred, Pdyn, seed);
    float* s_obs = calloc((size_t)G * Tm * OS, 4); int32_t* s_act = calloc((size_t)G * Tm, 4);
    int* s_len = calloc(G, sizeof(int));
    OTTT* env = malloc(sizeof(OTTT) * G);
    for (int g = 0; g < G; ++g) ttt_reset(&env[g]);
    float stacked[1024];
    for (int k = 0; k < 4; ++k) tally[k] = 0;
    for (int mv = 0; mv < moves; ++mv) {
        const uint32_t step = move0 + (uint32_t)mv;
        for (int g = 0; g < G; ++g) {
            const int T = s_len[g];
            float* oh = s_obs + (size_t)g * Tm * OS;
            for (int i = 0; i < OS; ++i) oh[(size_t)T * OS + i] = (float)env[g].b[i];
            uint8_t legal[MAXA]; ttt_legal(&env[g], legal);
            const int p = env[g].player;
            const uint32_t gid = game_offset + (uint32_t)g;
            int a;
            if (!random_opponent || p == muzero_player) {               /* :357-358 */
                ora_stacked_obs(c, oh, s_act + (size_t)g * Tm, T + 1, stacked);
                int root = run_mcts(&X, stacked, legal, p, 1, gid, step, NULL);
                a = select_action(&X, root, temperature, gid, step) + 1;
            } else {                                                    /* :360, :321 */
                int acts[MAXA], n = 0;
                for (int b = 0; b < A; ++b) if (legal[b]) acts[n++] = b;
                a = acts[mz_rng_below(mz_rng_u32(seed, MZ_RNG_OPPONENT, gid, step, 0), (uint32_t)n)] + 1;
            }
            ttt_step(&env[g], a);
            float r = ttt_reward(&env[g], p);
            int done = ttt_terminated(&env[g]);
            s_act[(size_t)g * Tm + T] = a;
            s_len[g] = T + 1;
            if (done || s_len[g] > c->max_moves) {
                int w = r == 0.0f ? 0 : 3 - p;
                tally[0] += 1;
                tally[w == 0 ? 3 : w == muzero_player ? 1 : 2] += 1;
                s_len[g] = 0; ttt_reset(&env[g]);
            }
        }
    }
    for (int g = 0; g < G; ++g) {
        slot_len[g] = s_len[g]; slot_player[g] = env[g].player;
        memcpy(slot_board + (size_t)g * OS, env[g].b, OS);
    }
    ctx_free(&X);
    free(s_obs); free(s_act); free(s_len); free(env);
    return 0;
}

/* ================================================== actor–learner loop
 * self_play! (SelfPlay.jl:384-419) ‖ learning! (Learning.jl:306-438), the
 * coupling of quirk Q16 restated deterministically for G lockstep self-play
 * slots — the schedule of the engine's mz_train_run:
 *   1. one move of every slot (play_game's loop body, SelfPlay.jl:343-380)
 *      with the ACTOR's nets: move key move0 + m, game id game_offset + g,
 *      temperature visit_softmax_temperature_fn(t) (:48-56, t = learner steps
 *      so far) taken at the game's first move and kept to its end (play_game
 *      takes T once per game, :396-407), 0 once a game has
 *      temperature_threshold moves (:344-346);
 *   2. the games that ended are saved in slot order (save_game,
 *      ReplayBuffer.jl:133-161, FIFO of `cap` games) and their slots restart;
 *   3. one learner step per saved game (self_play! take!s training_step once
 *      per game, :396; learning! put!s once per step, Learning.jl:411) while
 *      t <= training_steps (:327): get_batch keyed by step t+1, the
 *      ref_semantics step with eta = Cos(t+1); t += 1;
 *   4. after step t with t % checkpoint_interval == 0 && t > 1 the actor
 *      takes the queued nets and the learner's nets of step t are queued
 *      (remote_NNs is a capacity-1 channel that starts with the initial nets,
 *      only fetch()ed by self-play, :392, 399-401; Learning.jl:416-418): the
 *      actor runs one checkpoint behind.
 * TicTacToe only (the oracle's env).  P{l,a,q}[3]: learner / actor / queued
 * nets, updated in place; the learner's ADAM state m, v, bp as in
 * ora_learner_step.  Outputs: t (in/out), counters {num_played_games,
 * num_played_steps, total_samples}, the held games (oldest first: T, obs
 * (27,T), actions, rewards, to_play, child visits (A,T), root values; each
 * sized for max_moves + 1 moves), the slots' move counts / boards / players,
 * the last step's losses.                                                   */
static double ora_temp_fn(int64_t t) { return t < 500000 ? 1.0 : t < 750000 ? 0.5 : 0.25; }

EXPORT int ora_train_loop(const mz_config* cin, const ora_nethp* hp, float* Pl0, float* Pl1, float* Pl2,
                          float* Pa0, float* Pa1, float* Pa2, float* Pq0, float* Pq1, float* Pq2,
                          float* m_all, float* v_all, double* bp, uint64_t seed, int G, int cap, int moves,
                          uint32_t move0, uint32_t game_offset, int64_t* t_io, int64_t* counters,
                          int32_t* held_T, float* held_obs, int32_t* held_act, float* held_rew,
                          int32_t* held_tp, float* held_cv, float* held_rv, int32_t* slot_len,
                          uint8_t* slot_board, int32_t* slot_player, float* losses) {
    mz_config c = *cin;
    const int A = c.action_space_size, Tm = c.max_moves + 1, OS = 27, B = c.batch_size, K = c.num_unroll_steps;
    if (c.observation_shape[0] * c.observation_shape[1] * c.observation_shape[2] != OS || A != 9) return -1;
    const size_t n0 = ora_param_count(&c, hp, MZ_NET_REPR), n1 = ora_param_count(&c, hp, MZ_NET_PRED),
                 n2 = ora_param_count(&c, hp, MZ_NET_DYN);
    OCtx X; ctx_init(&X, &c, hp, Pa0, Pa1, Pa2, seed);
    /* games in progress and the ring, (27,T) float observations as OHist wants */
    float* s_obs = calloc((size_t)G * Tm * OS, 4); int32_t* s_act = calloc((size_t)G * Tm, 4);
    float* s_rew = calloc((size_t)G * Tm, 4); int32_t* s_tp = calloc((size_t)G * Tm, 4);
    float* s_cv = calloc((size_t)G * Tm * A, 4); float* s_rv = calloc((size_t)G * Tm, 4);
    int* s_len = calloc(G, sizeof(int));
    float* s_temp = calloc(G, sizeof(float));
    OTTT* env = malloc(sizeof(OTTT) * G);
    for (int g = 0; g < G; ++g) ttt_reset(&env[g]);
    float* r_obs = calloc((size_t)cap * Tm * OS, 4); int32_t* r_act = calloc((size_t)cap * Tm, 4);
    float* r_rew = calloc((size_t)cap * Tm, 4); int32_t* r_tp = calloc((size_t)cap * Tm, 4);
    float* r_cv = calloc((size_t)cap * Tm * A, 4); float* r_rv = calloc((size_t)cap * Tm, 4);
    int* r_len = calloc(cap, sizeof(int));
    int64_t played = 0, steps = 0, samples = 0, t = *t_io;
    int osz = c.observation_shape[0] * c.observation_shape[1] *
              (c.observation_shape[2] * (c.stacked_observations + 1) + c.stacked_observations);
    float* b_obs = malloc(sizeof(float) * (size_t)B * osz); float* b_act = malloc(sizeof(float) * B * (K + 1));
    float* b_tv = malloc(sizeof(float) * B * (K + 1)); float* b_tr = malloc(sizeof(float) * B * (K + 1));
    float* b_tp = malloc(sizeof(float) * (size_t)B * (K + 1) * A); float* b_gs = malloc(sizeof(float) * B);
    int32_t* b_idx = malloc(sizeof(int32_t) * 2 * B);
    OHist* hist = malloc(sizeof(OHist) * cap);
    float stacked[1024];
    int* fin = malloc(sizeof(int) * G);
    for (int mv = 0; mv < moves; ++mv) {
        const uint32_t step = move0 + (uint32_t)mv;
        int nfin = 0;
        for (int g = 0; g < G; ++g) {                                   /* 1. one move per slot */
            const int T = s_len[g];
            float* oh = s_obs + (size_t)g * Tm * OS;
            for (int i = 0; i < OS; ++i) oh[(size_t)T * OS + i] = (float)env[g].b[i];   /* :352 */
            ora_stacked_obs(&c, oh, s_act + (size_t)g * Tm, T + 1, stacked);           /* :355 */
            uint8_t legal[MAXA]; ttt_legal(&env[g], legal);
            const int p = env[g].player;                                /* :351 */
            if (T == 0) s_temp[g] = (float)ora_temp_fn(t);   /* one temperature per game, :396-407 */
            float temp = s_temp[g];
            if (c.temperature_threshold >= 0 && T >= c.temperature_threshold) temp = 0.0f;   /* :344-346 */
            const uint32_t gid = game_offset + (uint32_t)g;
            int root = run_mcts(&X, stacked, legal, p, 1, gid, step, NULL);               /* :359 */
            int a = select_action(&X, root, temp, gid, step) + 1;       /* :360 */
            ttt_step(&env[g], a);                                       /* :366 */
            float r = ttt_reward(&env[g], p);                           /* :367 */
            int done = ttt_terminated(&env[g]);                         /* :368 */
            search_stats(&X, root, s_cv + ((size_t)g * Tm + T) * A, s_rv + (size_t)g * Tm + T);   /* :375 */
            s_act[(size_t)g * Tm + T] = a; s_rew[(size_t)g * Tm + T] = r; s_tp[(size_t)g * Tm + T] = p;
            s_len[g] = T + 1;
            if (done || s_len[g] > c.max_moves) fin[nfin++] = g;        /* :343 */
        }
        for (int k = 0; k < nfin; ++k) {                                /* 2. save_game, slot order */
            const int g = fin[k], T = s_len[g];
            played += 1; steps += T; samples += T;
            const int slot = (int)((played - 1) % cap);
            if (played > cap) samples -= r_len[slot];                   /* FIFO eviction, :158 */
            r_len[slot] = T;
            memcpy(r_obs + (size_t)slot * Tm * OS, s_obs + (size_t)g * Tm * OS, sizeof(float) * (size_t)T * OS);
            memcpy(r_act + (size_t)slot * Tm, s_act + (size_t)g * Tm, 4 * (size_t)T);
            memcpy(r_rew + (size_t)slot * Tm, s_rew + (size_t)g * Tm, 4 * (size_t)T);
            memcpy(r_tp + (size_t)slot * Tm, s_tp + (size_t)g * Tm, 4 * (size_t)T);
            memcpy(r_cv + (size_t)slot * Tm * A, s_cv + (size_t)g * Tm * A, 4 * (size_t)T * A);
            memcpy(r_rv + (size_t)slot * Tm, s_rv + (size_t)g * Tm, 4 * (size_t)T);
            s_len[g] = 0; ttt_reset(&env[g]);
        }
        for (int k = 0; k < nfin; ++k) {                                /* 3. one learner step per game */
            if (t > c.training_steps) break;                            /* while t <= training_steps */
            const int nh = (int)(played < cap ? played : cap);
            const int64_t oldest = played - nh + 1;
            for (int i = 0; i < nh; ++i) {
                const int slot = (int)((oldest + i - 1) % cap);
                hist[i] = (OHist){r_len[slot], r_obs + (size_t)slot * Tm * OS, r_act + (size_t)slot * Tm,
                                  r_rew + (size_t)slot * Tm, r_tp + (size_t)slot * Tm,
                                  r_cv + (size_t)slot * Tm * A, r_rv + (size_t)slot * Tm};
            }
            const uint32_t st = (uint32_t)(t + 1);
            ora_get_batch(&c, hist, nh, (int)oldest, seed, st, b_obs, b_act, b_tv, b_tr, b_tp, b_gs, b_idx);
            ora_learner_step(&c, hp, Pl0, Pl1, Pl2, m_all, v_all, bp, B, b_obs, b_act, b_tv, b_tp, b_gs,
                             ora_cos_schedule(1e-4, 1e-1, 10, (int)st), losses);
            t = st;
            if (t % c.checkpoint_interval == 0 && t > 1) {              /* 4. actor <- queued, queue <- learner */
                memcpy(Pa0, Pq0, 4 * n0); memcpy(Pa1, Pq1, 4 * n1); memcpy(Pa2, Pq2, 4 * n2);
                memcpy(Pq0, Pl0, 4 * n0); memcpy(Pq1, Pl1, 4 * n1); memcpy(Pq2, Pl2, 4 * n2);
            }
        }
    }
    *t_io = t;
    counters[0] = played; counters[1] = steps; counters[2] = samples;
    const int nh = (int)(played < cap ? played : cap);
    for (int i = 0; i < nh; ++i) {                                      /* held games, oldest first */
        const int slot = (int)((played - nh + i) % cap), T = r_len[slot];
        held_T[i] = T;
        memcpy(held_obs + (size_t)i * Tm * OS, r_obs + (size_t)slot * Tm * OS, sizeof(float) * (size_t)T * OS);
        memcpy(held_act + (size_t)i * Tm, r_act + (size_t)slot * Tm, 4 * (size_t)T);
        memcpy(held_rew + (size_t)i * Tm, r_rew + (size_t)slot * Tm, 4 * (size_t)T);
        memcpy(held_tp + (size_t)i * Tm, r_tp + (size_t)slot * Tm, 4 * (size_t)T);
        memcpy(held_cv + (size_t)i * Tm * A, r_cv + (size_t)slot * Tm * A, 4 * (size_t)T * A);
        memcpy(held_rv + (size_t)i * Tm, r_rv + (size_t)slot * Tm, 4 * (size_t)T);
    }
    for (int g = 0; g < G; ++g) {
        slot_len[g] = s_len[g]; slot_player[g] = env[g].player;
        memcpy(slot_board + (size_t)g * OS, env[g].b, OS);
    }
    ctx_free(&X);
    free(s_obs); free(s_act); free(s_rew); free(s_tp); free(s_cv); free(s_rv); free(s_len); free(s_temp); free(env);
    free(r_obs); free(r_act); free(r_rew); free(r_tp); free(r_cv); free(r_rv); free(r_len);
    free(b_obs); free(b_act); free(b_tv); free(b_tr); free(b_tp); free(b_gs); free(b_idx); free(hist); free(fin);
    return nh;
}

/* ======================================================== detmath exports
 * for tests (accuracy vs libm) and the Python mirror */
EXPORT float ora_det_expf(float x) { return det_expf(x); }
EXPORT float ora_det_tanhf(float x) { return det_tanhf(x); }
EXPORT float ora_det_logf(float x) { return det_logf(x); }
EXPORT double ora_det_exp(double x) { return det_exp(x); }
EXPORT double ora_det_log(double x) { return det_log(x); }
EXPORT uint32_t ora_rng_u32(uint64_t seed, uint32_t purpose, uint32_t id, uint32_t step, uint32_t idx) {
    return mz_rng_u32(seed, purpose, id, step, idx);
}
EXPORT void ora_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out) {
    mz_u32x4 r = mz_philox(c0, c1, c2, c3, k0, k1);
    memcpy(out, r.v, 16);
}
EXPORT void ora_dirichlet(uint64_t seed, uint32_t game, uint32_t step, int n, float alpha, float* out) {
    mz_dirichlet(seed, game, step, n, alpha, out);
}
EXPORT void ora_softmax(const float* x, int n, float* y) { softmax_n(x, n, y); }
EXPORT float ora_dot(const float* Wcol, int out, int in, int o, const float* x) { return mz_dot(Wcol, out, in, o, x); }
