/* CPU AddressSanitizer / UBSan build of the oracle (oracle/mz_oracle.c, the
 * test infrastructure every parity claim rests on; SURVEY §5 "sanitizer
 * build of the host C/C++").  The oracle's source is compiled into this
 * driver as one translation unit with -fsanitize=address,undefined, and the
 * driver runs its main entry points on small cases: the whole actor-learner
 * loop (play_game, save_game FIFO, get_batch / make_target, the learner step
 * and ADAM, ora_train_loop), searches with tree dumps on the FC and ResNet
 * TicTacToe nets and the Connect4 FC net, PER sampling and priority updates,
 * evaluation play, and the Atari downsampler forward.  A sanitizer report
 * aborts; exit 0 = clean.  Built and run by tests/test_sanitizers.py. */
#include "../../oracle/mz_oracle.c"

#include <stdio.h>

static uint32_t lcg = 12345u;
static float frand(void) { lcg = lcg * 1664525u + 1013904223u; return ((float)(lcg >> 8) / 16777216.0f - 0.5f); }

static mz_config ttt_conf(int sims) {
    mz_config c; memset(&c, 0, sizeof(c));
    c.seed = 1337; c.observation_shape[0] = 3; c.observation_shape[1] = 3; c.observation_shape[2] = 3;
    c.action_space_size = 9; c.players = 2; c.stacked_observations = 1; c.muzero_player = 1;
    c.num_workers = 1; c.max_moves = 9; c.temperature_threshold = -1; c.dirichlet_alpha = 0.25f;
    c.exploration_eps = 0.25f; c.pb_c_base = 19652; c.pb_c_init = 1.25f; c.discount = 0.997f;
    c.num_iters = sims; c.replay_buffer_size = 16; c.num_unroll_steps = 5; c.td_steps = 5;
    c.PER = 0; c.PER_alpha = 1; c.training_steps = 1000; c.batch_size = 8; c.checkpoint_interval = 5;
    c.value_loss_weight = 0.25f;
    return c;
}
static ora_nethp fc_hp(int hidden) {
    ora_nethp h; memset(&h, 0, sizeof(h));
    h.kind = 0; h.ff.width_hidden = 64; h.ff.depth_representation = 3; h.ff.depth_prediction = 3;
    h.ff.depth_dynamics = 3; h.ff.depth_policy = 1; h.ff.depth_value = 1; h.ff.depth_reward = 1;
    h.ff.depth_state_head = 3; h.ff.batch_norm_momentum = 0.6f; h.ff.hidden_state_size = hidden;
    h.ff.reward_activation = MZ_ACT_TANH;
    return h;
}
static ora_nethp rn_hp(int ds) {
    ora_nethp h; memset(&h, 0, sizeof(h));
    h.kind = 1; h.rn.num_blocks = 2; h.rn.num_filters = ds ? 16 : 64; h.rn.conv_kernel_size[0] = 3;
    h.rn.conv_kernel_size[1] = 3; h.rn.num_second_head_filters = 2; h.rn.num_first_head_filters = 1;
    h.rn.batch_norm_momentum = 0.6f; h.rn.downsample = ds; h.rn.depth_policy = 1; h.rn.depth_value = 1;
    h.rn.width_hidden = 64; h.rn.reward_activation = MZ_ACT_TANH;
    return h;
}
static float* params(const mz_config* c, const ora_nethp* h, int net, float scale) {
    size_t n = ora_param_count(c, h, net);
    float* p = malloc(sizeof(float) * n);
    for (size_t i = 0; i < n; ++i) p[i] = scale * frand();
    return p;
}

static void search(const mz_config* c, const ora_nethp* hp, int G, int feat) {
    const int A = c->action_space_size, S = c->num_iters;
    float *P0 = params(c, hp, 0, 0.2f), *P1 = params(c, hp, 1, 0.2f), *P2 = params(c, hp, 2, 0.2f);
    float* obs = malloc(sizeof(float) * (size_t)G * feat);
    uint8_t* legal = malloc((size_t)G * A);
    int32_t* tp = malloc(sizeof(int32_t) * G);
    for (int i = 0; i < G * feat; ++i) obs[i] = frand() > 0.1f ? 1.0f : 0.0f;
    for (int g = 0; g < G; ++g) {
        for (int a = 0; a < A; ++a) legal[g * A + a] = frand() > -0.2f;
        legal[g * A + (g % A)] = 1;
        tp[g] = 1 + g % c->players;
    }
    if (G > 1) { memset(legal + A, 0, A); legal[A + 2] = 1; }          /* one legal action: a deep chain */
    float *cv = malloc(sizeof(float) * G * A), *rv = malloc(sizeof(float) * G);
    int32_t* act = malloc(sizeof(int32_t) * G);
    const size_t E = (size_t)G * (S + 1) * A;
    int32_t *eN = malloc(4 * E), *ech = malloc(4 * E), *ntp = malloc(4 * (size_t)G * (S + 1));
    float *eW = malloc(4 * E), *eP = malloc(4 * E), *eR = malloc(4 * E);
    int64_t stats[2] = {0, 0};
    for (int explore = 0; explore < 2; ++explore)
        ora_mcts_search(c, hp, P0, P1, P2, 7, G, obs, legal, tp, explore, 3, 11, explore ? 1.0f : 0.0f, cv, rv,
                        act, eN, eW, eP, eR, ech, ntp, stats);
    for (int g = 0; g < G; ++g)
        if (act[g] < 1 || act[g] > A) { fprintf(stderr, "bad action\n"); exit(1); }
    free(P0); free(P1); free(P2); free(obs); free(legal); free(tp); free(cv); free(rv); free(act);
    free(eN); free(ech); free(ntp); free(eW); free(eP); free(eR);
}

int main(void) {
    /* 1. the actor-learner loop on the FC TicTacToe nets (ora_train_loop) */
    {
        mz_config c = ttt_conf(8);
        ora_nethp hp = fc_hp(27);
        const int G = 4, cap = 8, moves = 40, Tm = c.max_moves + 1, A = 9;
        size_t n[3];
        float *Pl[3], *Pa[3], *Pq[3];
        size_t ntot = 0;
        for (int k = 0; k < 3; ++k) {
            n[k] = ora_param_count(&c, &hp, k); ntot += n[k];
            Pl[k] = params(&c, &hp, k, 0.3f);
            Pa[k] = malloc(4 * n[k]); Pq[k] = malloc(4 * n[k]);
            memcpy(Pa[k], Pl[k], 4 * n[k]); memcpy(Pq[k], Pl[k], 4 * n[k]);
        }
        float *m = calloc(ntot, 4), *v = calloc(ntot, 4);
        double bp[2] = {0.9, 0.999};
        int64_t t = 0, counters[3];
        int32_t *hT = malloc(4 * cap), *hact = malloc(4 * (size_t)cap * Tm), *htp = malloc(4 * (size_t)cap * Tm);
        float *hobs = malloc(4 * (size_t)cap * Tm * 27), *hrew = malloc(4 * (size_t)cap * Tm);
        float *hcv = malloc(4 * (size_t)cap * Tm * A), *hrv = malloc(4 * (size_t)cap * Tm);
        int32_t *slen = malloc(4 * G), *spl = malloc(4 * G);
        uint8_t* sb = malloc((size_t)G * 27);
        float losses[8];
        int nh = ora_train_loop(&c, &hp, Pl[0], Pl[1], Pl[2], Pa[0], Pa[1], Pa[2], Pq[0], Pq[1], Pq[2], m, v, bp,
                                9, G, cap, moves, 100, 4, &t, counters, hT, hobs, hact, hrew, htp, hcv, hrv, slen,
                                sb, spl, losses);
        printf("train_loop: %d games held, %lld learner steps, %lld played\n", nh, (long long)t,
               (long long)counters[0]);
        if (nh <= 0 || t <= 0) { fprintf(stderr, "train loop made no progress\n"); return 1; }
        /* 2. PER over the held games: init, prioritized batch, update */
        OHist* hist = malloc(sizeof(OHist) * nh);
        int total = 0;
        for (int i = 0; i < nh; ++i) {
            hist[i] = (OHist){hT[i], hobs + (size_t)i * Tm * 27, hact + (size_t)i * Tm, hrew + (size_t)i * Tm,
                              htp + (size_t)i * Tm, hcv + (size_t)i * Tm * A, hrv + (size_t)i * Tm};
            total += hT[i];
        }
        float* prio = calloc((size_t)nh * Tm, 4);
        float* gprio = calloc(nh, 4);
        int32_t* lens = malloc(4 * nh);
        for (int i = 0; i < nh; ++i) { ora_per_init(&c, &hist[i], prio + (size_t)i * Tm, gprio + i); lens[i] = hT[i]; }
        const int B = c.batch_size, K = c.num_unroll_steps, osz = 63;
        float *bo = malloc(4 * (size_t)B * osz), *ba = malloc(4 * B * (K + 1)), *btv = malloc(4 * B * (K + 1));
        float *btr = malloc(4 * B * (K + 1)), *btp = malloc(4 * (size_t)B * (K + 1) * A), *bgs = malloc(4 * B);
        float* bw = malloc(4 * B);
        int32_t* bidx = malloc(8 * B);
        ora_get_batch_per(&c, hist, prio, gprio, nh, Tm, 1, 9, 5, bo, ba, btv, btr, btp, bgs, bw, bidx);
        float* pv = malloc(4 * B * (K + 1));
        for (int i = 0; i < B * (K + 1); ++i) pv[i] = frand();
        ora_update_priorities(&c, prio, gprio, lens, nh, Tm, 1, B, bidx, pv, btv);
        ora_get_batch(&c, hist, nh, 1, 9, 6, bo, ba, btv, btr, btp, bgs, bidx);
        free(hist); free(prio); free(gprio); free(lens); free(bo); free(ba); free(btv); free(btr); free(btp);
        free(bgs); free(bw); free(bidx); free(pv);
        for (int k = 0; k < 3; ++k) { free(Pl[k]); free(Pa[k]); free(Pq[k]); }
        free(m); free(v); free(hT); free(hact); free(htp); free(hobs); free(hrew); free(hcv); free(hrv);
        free(slen); free(spl); free(sb);
    }
    /* 3. searches: FC and ResNet TicTacToe, Connect4 FC (6x7, 7 actions) */
    {
        mz_config c = ttt_conf(20);
        ora_nethp f = fc_hp(27), r = rn_hp(0);
        search(&c, &f, 5, 63);
        c.num_iters = 6;
        search(&c, &r, 3, 63);
        mz_config c4 = ttt_conf(12);
        c4.observation_shape[0] = 6; c4.observation_shape[1] = 7; c4.action_space_size = 7; c4.max_moves = 42;
        ora_nethp f4 = fc_hp(126);
        search(&c4, &f4, 3, 6 * 7 * 7);
    }
    /* 4. the Atari downsampler forward (84x84x4 -> 6x6) */
    {
        mz_config c = ttt_conf(2);
        c.observation_shape[0] = 84; c.observation_shape[1] = 84; c.observation_shape[2] = 4;
        c.action_space_size = 18; c.players = 1; c.stacked_observations = 0;
        ora_nethp r = rn_hp(1);
        float* P0 = params(&c, &r, 0, 0.05f);
        const int feat = 84 * 84 * 4;
        float* x = malloc(4 * (size_t)feat);
        for (int i = 0; i < feat; ++i) x[i] = frand() + 0.5f;
        const int H = ora_hidden_size(&c, &r);
        float* out = malloc(4 * (size_t)H);
        ora_net_forward(&c, &r, MZ_NET_REPR, P0, x, 1, out, NULL);
        printf("downsampler forward: hidden %d\n", H);
        free(P0); free(x); free(out);
    }
    printf("oracle_asan: clean\n");
    return 0;
}
