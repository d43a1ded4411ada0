/*
 * mz.h — C ABI of libmz, the MI355X-native MuZero self-play + learner engine.
 *
 * This is the drop-in boundary for the reference's hot path.
 * The reference (deveshjawla/MuZero.jl) is Julia; a maintainer binds these
 * symbols with `ccall`; tests bind them with ctypes.
 *
 * Conventions (SURVEY §8b "Conventions"):
 *   - every entry point returns int status: 0 = OK, < 0 = error; the message
 *     is in mz_last_error(h) (the reference raises Julia exceptions / @assert,
 *     e.g. src/SelfPlay.jl:243-244);
 *   - host buffers are caller-owned and borrowed for the duration of the call;
 *     `_dev` variants take device pointers and a hipStream_t (as void*);
 *   - one handle per GPU, one host thread per handle; calls are synchronous
 *     at return (the `_dev` variants are stream-ordered instead); a
 *     host-synchronous call (weights, state, checkpoints, replay / debug
 *     read-outs, the host-buffer search and learner step) first waits for all
 *     of the process's work on the device, so `_dev` work queued on a caller
 *     stream is complete before it reads or overwrites engine memory
 *     (mz_set_sync_stream narrows that wait to one caller stream);
 *   - action ids are 1-based (Julia convention), arrays are column-major with
 *     the reference's shapes (W,H,C,N): feature index = w + W*h + W*H*c.
 */
#ifndef MZ_H
#define MZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MZ_MAX_ACTIONS 32

/* Config — field names and defaults of src/Constructors.jl:18-52.
 * Julia `dirichlet_α`/`exploration_ϵ` are spelled dirichlet_alpha /
 * exploration_eps; `temperature_threshold = nothing` is -1; `action_space`
 * is 1:action_space_size; `players` is 1:players.                         */
typedef struct mz_config {
    int32_t seed;                    /* 1337 (Constructors.jl:19, never used by the reference) */
    int32_t observation_shape[3];    /* (W,H,C) per observation, e.g. (3,3,3) */
    int32_t action_space_size;       /* |action_space| = 9 for TicTacToe */
    int32_t players;                 /* |players| = 2 */
    int32_t stacked_observations;    /* 1 */
    int32_t muzero_player;           /* 1 */
    int32_t intermediate_rewards;    /* false */
    int32_t num_workers;
    int32_t selfplay_on_gpu;
    int32_t max_moves;               /* 9 */
    int32_t temperature_threshold;   /* -1 = nothing */
    float dirichlet_alpha;           /* 0.25 */
    float exploration_eps;           /* 0.25 */
    int32_t pb_c_base;               /* 19652 */
    float pb_c_init;                 /* 1.25 */
    float discount;                  /* 0.997 */
    int32_t num_iters;               /* simulations per move */
    int32_t replay_buffer_size;      /* 10000 */
    int32_t num_unroll_steps;        /* K = 5 */
    int32_t td_steps;                /* 5 */
    int32_t PER;                     /* false */
    int32_t PER_alpha;               /* 1 */
    int32_t training_steps;          /* 10000 */
    int32_t batch_size;              /* 32 */
    int32_t checkpoint_interval;     /* 10 */
    float value_loss_weight;         /* 0.25 (never applied by the reference, Q11) */
} mz_config;

enum { MZ_ACT_IDENTITY = 0, MZ_ACT_RELU = 1, MZ_ACT_TANH = 2 };

/* FeedForwardHP — src/Constructors.jl:62-75 */
typedef struct mz_ffhp {
    int32_t width_hidden;            /* 64 */
    int32_t depth_representation;    /* 3 */
    int32_t depth_prediction;        /* 3 */
    int32_t depth_dynamics;          /* 3 */
    int32_t depth_policy;            /* 1 */
    int32_t depth_value;             /* 1 */
    int32_t depth_reward;            /* 1 */
    int32_t depth_state_head;        /* 3 */
    int32_t use_batch_norm;          /* false; true: make_dense = Dense then BatchNorm(out, relu) in test mode (Learning.jl:70-78) */
    float batch_norm_momentum;       /* 0.6 */
    int32_t hidden_state_size;       /* 27 = prod(observation_shape) */
    int32_t reward_activation;       /* MZ_ACT_TANH */
} mz_ffhp;

/* ResNetHP — src/Constructors.jl:77-90, the residual conv towers of
 * Learning.jl:148-255.  The reference's ResNet constructors cannot run
 * (SURVEY §2.1 Q12); the engine builds their intended architecture
 * (DESIGN.md §9): stride-1 zero-padded Conv (Flux convolution, kernel
 * flipped), BatchNorm in test mode (the reference's forward runs outside the
 * pullback) with its running statistics, residual blocks
 * conv-BN-relu-conv-BN-(+x)-relu, 1x1 convs in prediction / dynamics, and the
 * heads' Dense layers of width `width_hidden` (a field the reference reads
 * from ResNetHP but never declares).                                       */
typedef struct mz_resnet_hp {
    int32_t num_blocks;              /* residual blocks per tower */
    int32_t num_filters;             /* nf */
    int32_t conv_kernel_size[2];     /* representation kernel (odd), e.g. (3,3) */
    int32_t num_second_head_filters; /* 2: policy head 1x1 conv channels */
    int32_t num_first_head_filters;  /* 1: value / reward head 1x1 conv channels */
    float batch_norm_momentum;       /* 0.6 (unused in test mode) */
    int32_t downsample;              /* false; true = the Atari downsampler of Learning.jl:175-187
                                        (BASELINE configs[4]): Conv(k, C=>C, stride 2), 2 blocks,
                                        Conv(k, C=>2C, stride 2), 3 blocks, MeanPool((3,3), stride 2,
                                        pad 1), 3 blocks, MeanPool, then the representation's
                                        Conv(k, 2C=>nf) + blocks: 84x84 -> 6x6.  The hidden board
                                        (representation_output_size) is then 6x6, and the
                                        downsampler's params lead the representation's Flux.params */
    int32_t depth_policy;            /* hidden Dense layers (the reference reuses depth_value, kept) */
    int32_t depth_value;             /* hidden Dense layers of the value / reward / policy heads */
    int32_t width_hidden;            /* 64: Dense width of the heads */
    int32_t reward_activation;       /* MZ_ACT_TANH */
} mz_resnet_hp;

/* The three networks of the `NNs` NamedTuple (SelfPlay.jl:230). */
enum { MZ_NET_REPR = 0, MZ_NET_PRED = 1, MZ_NET_DYN = 2 };

typedef struct mz_handle mz_handle;

/* Create an engine on HIP device `device` (replaces init_* + the Julia
 * process setup of games/tictactoe/main.jl:15-28).  `max_games` bounds the
 * batch G of mz_mcts_search; `rng_seed` keys every Philox stream.         */
int mz_engine_create(const mz_config* conf, const mz_ffhp* hyper, int device,
                     int max_games, uint64_t rng_seed, mz_handle** out);
/* Same engine with the ResNet networks (ResNetHP, configs 3-5).  Hidden
 * state = (W, H, num_filters) on the observation board (W, H), or on the
 * downsampled board with ResNetHP.downsample; the dynamics input is
 * (W, H, num_filters+1).  action_space_size <= 32 (the FC engine: <= 16). */
int mz_engine_create_resnet(const mz_config* conf, const mz_resnet_hp* hyper, int device,
                            int max_games, uint64_t rng_seed, mz_handle** out);
void mz_engine_destroy(mz_handle* h);
const char* mz_last_error(const mz_handle* h);
/* message of the last failed mz_engine_create (no handle exists then) */
const char* mz_create_error(void);

/* Parameter counts and exchange in Flux order: for every Dense, W (out,in)
 * column-major then b; Chain order, Split paths in order
 * (Learning.jl:87-142).  FC TicTacToe: 18331 / 23242 / 33308 floats.      */
int mz_net_param_count(const mz_handle* h, int net, size_t* n);
int mz_weights_set(mz_handle* h, int net, const float* flat, size_t n);
int mz_weights_get(mz_handle* h, int net, float* flat, size_t n);

/* Batched forward of one net (the Flux Chain call, Learning.jl:87-142).
 *   REPR: x = stacked obs (W,H,Cs,n) -> out0 = h (hidden,n)
 *   PRED: x = h (hidden,n)          -> out0 = value (1,n), out1 = policy probs (A,n)
 *   DYN : x = state-action (W,H,C+1,n) -> out0 = h' (hidden,n), out1 = reward (1,n) */
int mz_net_forward(mz_handle* h, int net, const float* x, int n, float* out0, float* out1);

/* Batched run_mcts + select_action + store_search_stats! for G games
 * (SelfPlay.jl:230-306, 115-122).
 *   obs        (W,H,Cs,G) stacked observations (get_stacked_observations)
 *   legal_mask (A,G) uint8, nonzero = legal (legal_action_space), >= 1 per game
 *   to_play    (G) current player, 1-based
 *   exploration  add Dirichlet noise at the root (SelfPlay.jl:247-249)
 *   rng_step   move counter keying the Philox streams; game_offset = global id
 *              of game 0 (shard offset on multi-GPU)
 *   temperature  visit_softmax_temperature (0 = argmax, INFINITY = uniform)
 * outputs: child_visits (A,G) = N_a / sum N, root_value (G) = node_value(root),
 *          action_out (G) in 1..A.                                         */
int mz_mcts_search(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask,
                   const int32_t* to_play, int exploration, uint32_t rng_step,
                   uint32_t game_offset, float temperature,
                   float* child_visits, float* root_value, int32_t* action_out);

/* Same, all buffers in device memory, stream-ordered on `stream` (hipStream_t). */
int mz_mcts_search_dev(mz_handle* h, int G, const float* obs, const uint8_t* legal_mask,
                       const int32_t* to_play, int exploration, uint32_t rng_step,
                       uint32_t game_offset, float temperature,
                       float* child_visits, float* root_value, int32_t* action_out,
                       void* stream);

/* Host-synchronous calls wait for ALL of the process's device work by
 * default (hipDeviceSynchronize), which is always safe.  A caller that
 * orders its own `_dev` work can narrow that wait with narrow = 1: the calls
 * then wait only for `stream` (a hipStream_t as void*; NULL = the legacy
 * default stream) and the handle's own stream.  narrow = 0 restores the
 * device-wide wait.                                                        */
int mz_set_sync_stream(mz_handle* h, void* stream, int narrow);

/* Debug/parity: flags & 1 = keep a copy of every search's final tree in HBM
 * (the LDS-resident tree is otherwise discarded at kernel exit); flags & 2 =
 * time the ResNet search's network launches, flags & 4 = the ResNet
 * learner's unroll launches and the unroll launch of each
 * mz_learner_train_multi_dev (mz_learn_multi*) (mz_debug_kernel_time). */
int mz_debug_enable(mz_handle* h, int flags);

/* Debug/parity: copy the last search's tree statistics to host.  Per game,
 * expanded-node slots e = 0..S (0 = root, e = s+1 expanded by simulation s)
 * and child slots a = 0..A-1:
 *   edge_N/edge_W/edge_P/edge_R: (A, S+1, G), edge_child: expanded slot or -1,
 *   node_to_play (S+1, G); any pointer may be NULL.                        */
int mz_debug_tree(mz_handle* h, int G, int32_t* edge_N, float* edge_W, float* edge_P,
                  float* edge_R, int32_t* edge_child, int32_t* node_to_play);

/* Measurement: with mz_debug_enable(h, 2) every network launch of the
 * ResNet search (mz_rsearch_nets, its dominant kernel), with flag 4 every
 * learner unroll launch (mz_runroll_kernel, mz_learn_multi*), is bracketed by HIP events on
 * its stream; this returns the summed duration and the launch count since
 * the previous call, and resets them.                                      */
int mz_debug_kernel_time(mz_handle* h, double* total_ms, int* launches);

/* Debug/parity: the last learner unroll's read-outs (Learning.jl:347-370)
 * for its first B samples: values (K+1, B) and rewards (K+1, B) after their
 * activations, policies (A, K+1, B) as probabilities — the predictions the
 * loss reads (Q10 alignment: step 0 and step 1 both predict from h0,
 * reward 0 at step 0).  Any pointer may be NULL.                          */
int mz_debug_unroll(mz_handle* h, int B, float* values, float* policies, float* rewards);
/* The same read-outs of step step0 + i of the last mz_learner_train_multi_dev
 * that ran its multi-step form, 0 <= i < L; the per-step scratch is a ring of
 * at least 33 steps (the largest multiple of the chain-launch length <= 64),
 * so steps older than that are refused.                                     */
int mz_debug_unroll_step(mz_handle* h, int i, int B, float* values, float* policies, float* rewards);

/* One learner batch, the tuple returned by get_batch (ReplayBuffer.jl:216),
 * column-major as in the reference:
 *   observation (W,H,Cs,B), actions (K+1,B) as float action ids,
 *   target_values (K+1,B), target_rewards (K+1,B), target_policies (A,K+1,B),
 *   gradient_scale (B), weights (B): PER importance-sampling weights
 *   (weight_batch, ReplayBuffer.jl:211-215), NULL = all 1 (PER = false).     */
typedef struct mz_batch {
    int32_t batch_size;
    const float* observation;
    const float* actions;
    const float* target_values;
    const float* target_rewards;
    const float* target_policies;
    const float* gradient_scale;
    const float* weights;
} mz_batch;

/* Learner step in ref_semantics (Learning.jl:327-413, quirks Q10/Q11):
 * K-step unroll forward, losses, gradient 2θ, ADAM(β=(0.9,0.999), ϵ=1e-8)
 * with learning rate `eta` (the host evaluates Cos(λ0=1e-4, λ1=1e-1,
 * period=10) and passes it; Learning.jl:319,382).
 * losses_out[6] = {value, reward, policy, l2_repr, l2_pred, l2_dyn}; the
 * reference's three reported losses are value+reward+policy+l2_net.
 * Single-GPU form; data-parallel training uses the split form below.      */
int mz_learner_step(mz_handle* h, const mz_batch* batch, double eta, float* losses_out);

/* Learner mode.  MZ_LEARN_REF_SEMANTICS (default): the reference as written
 * — its pullbacks see only sum(sqnorm, params), so ∇ = 2θ (quirk Q11), and
 * the reported policy loss is Q11's broadcast.  MZ_LEARN_CORRECTED (every
 * net: FC with or without BatchNorm, ResNet with or without the downsampler): the loss
 * Learning.jl:261-288 means, differentiated through the unroll (real
 * backpropagation on MFMA, mz_backprop.hip), as a per-sample mean so a
 * data-parallel all-reduce-mean equals the global batch:
 *   L = (1/B) Σ_b (w_b/g_b) [Σ_k (v−z)² + Σ_k CE(logits, π) + ir·Σ_k (r−u)²] + Σθ²
 * (CE = logitcrossentropy on the policy head's logits).  Every learner entry
 * point follows the mode; losses_out = {value, reward, policy, Σθ² ×3}.    */
enum { MZ_LEARN_REF_SEMANTICS = 0, MZ_LEARN_CORRECTED = 1 };
int mz_learner_set_mode(mz_handle* h, int mode);

/* Split learner step for data-parallel training: (1) forward + losses +
 * the DATA TERM of the gradient into grad_dev (device, mz_grad_count
 * floats): ∂/∂θ of the loss without Σθ² — zero in ref_semantics (Q11),
 * the backpropagated term in the corrected mode; (2) the caller all-reduces
 * (sum) grad_dev across ranks; (3) mz_learner_apply_dev runs ADAM on
 * ∇ = grad_dev · grad_scale + 2θ (grad_scale = 1/world).  The rank-invariant
 * 2θ = ∂Σθ²/∂θ is added after the exchange, so the update equals the
 * single-GPU update bit for bit at every world size in ref_semantics (an
 * exchanged 2θ would be summed in f32 and round differently at world 8).
 * Stream-ordered on `stream`.                                              */
int mz_grad_count(const mz_handle* h, size_t* n);
int mz_learner_grad_dev(mz_handle* h, const mz_batch* dev_batch, float* grad_dev,
                        float* losses_dev, void* stream);
int mz_learner_apply_dev(mz_handle* h, const float* grad_dev, float grad_scale,
                         double eta, void* stream);

/* ---- Data-parallel learner over RCCL -------------------------
 * For hosts without torch.distributed (the Julia binding): one RCCL
 * communicator per handle, one handle per GPU.  Rank 0 calls
 * mz_dp_unique_id and hands the 128-byte id to every rank out of band (the
 * RemoteChannel / Distributed.jl of the reference host); each rank calls
 * mz_dp_init.  mz_dp_allreduce sums the gradient bucket (mz_grad_count
 * floats, grad_dev or the handle's gradient if NULL) in place over RCCL on
 * `stream`; mz_learner_train_dp = mz_learner_grad_sampled_dev (data term)
 * + that all-reduce + mz_learner_apply_dev(1/world, + 2θ).  librccl.so.1 is loaded on
 * first use (the copy already in the process if any).                      */
#define MZ_DP_ID_BYTES 128
int mz_dp_unique_id(uint8_t* id);
int mz_dp_init(mz_handle* h, int rank, int world, const uint8_t* id);
int mz_dp_allreduce(mz_handle* h, float* grad_dev, void* stream);
int mz_learner_train_dp(mz_handle* h, int32_t B, uint32_t step, double eta, float* losses_dev, void* stream);

/* ---- Device self-play and replay shard ------------
 * The loop body of play_game (SelfPlay.jl:330-382) and the replay buffer
 * (ReplayBuffer.jl) kept in HBM: no host round trip per move or per batch. */
enum { MZ_ENV_TICTACTOE = 0, MZ_ENV_CONNECT4 = 1, MZ_ENV_ATARI = 2 };

/* Device self-play state for G <= max_games game slots: env boards
 * (games/tictactoe/game.jl with quirk Q14, or the Connect4 env of BASELINE
 * configs[3], rules in muzero.jl_amd/games/connect4.py), each slot's
 * GameHistory (Constructors.jl:6-16) in HBM, and a replay shard: FIFO of
 * replay_games >= G finished games (ReplayBuffer.jl:133-161, PER = false;
 * the RemoteBufferChannel Dict keyed by game number).  Every slot starts a
 * new game.  The conf must match the env (TicTacToe (3,3,3)/9 actions,
 * Connect4 (6,7,3)/7 actions, the synthetic Atari-like env of configs[4]
 * (84,84,4)/18 actions with stacked_observations = 0: Philox-keyed frames,
 * rules in muzero.jl_amd/games/atari_synth.py; the records and the shard
 * hold one 84x84 byte frame per move and the observation is the env's
 * four-frame stack; its slots' initial games are drawn at the first
 * mz_selfplay_move, keyed by that move's global game ids game_offset + slot).
 * Calling it again discards the state.                                      */
int mz_selfplay_init(mz_handle* h, int env_kind, int G, int replay_games);

/* One move of every slot, on the device, stream-ordered: observation append
 * and stacked observations (SelfPlay.jl:351-355, Q15), legal mask, to_play,
 * the batched search (as mz_mcts_search_dev with exploration on), env step
 * and GameHistory append (:359-379).  Games that end (terminal, or more than
 * max_moves moves, :343) go to the replay shard in slot order (save_game)
 * and their slot starts a new game.  rng_step = the global move counter.   */
int mz_selfplay_move(mz_handle* h, uint32_t rng_step, uint32_t game_offset, float temperature,
                     void* stream);

/* Evaluation play (competitive_play!, SelfPlay.jl:421-435; play_game with
 * an opponent, :330-382; select_opponent_action, :311-325).  mode
 * MZ_SP_EVAL: finished games are not saved (competitive_play! keeps no
 * buffer) but tallied for mz_eval_results; with opponent MZ_OPP_RANDOM the
 * player != muzero_player (1 or 2) plays a uniform legal action (the Philox
 * OPPONENT stream keyed (game id, rng_step)) instead of the search's, the
 * intended reading of :321 (the reference reads `las`, defined only in the
 * "human" branch); MZ_OPP_SELF: MuZero plays both sides.  Pass
 * temperature 0 to mz_selfplay_move for competitive play.  MZ_SP_TRAIN
 * (default): self_play! (:384-419).  Applies to the following moves; the
 * games in progress continue.                                              */
enum { MZ_SP_TRAIN = 0, MZ_SP_EVAL = 1 };
enum { MZ_OPP_SELF = 0, MZ_OPP_RANDOM = 1 };
int mz_selfplay_mode(mz_handle* h, int mode, int opponent, int muzero_player);

/* Evaluation tally since mz_selfplay_init: {games finished, MuZero wins,
 * opponent wins, draws}; the winner is read from the last move's reward
 * (TicTacToe with quirk Q14: the player to move after it; Connect4: the
 * mover).  Synchronises.                                                    */
int mz_eval_results(mz_handle* h, int64_t* out4);

/* The shard's counters {num_played_games, num_played_steps, total_samples}
 * (ReplayBuffer.jl:133-161) and the games it holds; synchronises.          */
int mz_replay_counts(mz_handle* h, int64_t* counts, int32_t* games_in_buffer);

/* save_game of a host GameHistory of T moves (obs as 0/1 bytes (T, W*H*C),
 * actions / rewards / to_play / root_values (T), child_visits (A, T)).     */
int mz_replay_save_game(mz_handle* h, int32_t T, const uint8_t* obs, const int32_t* actions,
                        const float* rewards, const int32_t* to_play, const float* child_visits,
                        const float* root_values);

/* get_batch with make_target (ReplayBuffer.jl:5-50, 73-107, 188-217) on the
 * device: B samples drawn with the Philox streams of learner step `step`
 * (engine seed; sample_n_games uniform with replacement, sample_position
 * uniform, absorbing-state actions uniform).  Fills *batch with device
 * arrays owned by the handle (valid until the next call; feed them to
 * mz_learner_grad_dev) and, if index_batch != NULL, copies the (game
 * number, 1-based position) pairs to it (B x 2, synchronises).             */
int mz_replay_sample(mz_handle* h, int32_t B, uint32_t step, mz_batch* batch, int32_t* index_batch,
                     void* stream);

/* One learner iteration on a batch drawn from this GPU's replay shard:
 * get_batch (as mz_replay_sample(step)) + learning! (Learning.jl:327-404).
 * The sampling runs inside the FC unroll kernel (its own launch otherwise).
 * _grad_sampled_dev: results of mz_replay_sample + mz_learner_grad_dev (for
 * a gradient exchange before mz_learner_apply_dev).  _train_dev (one GPU,
 * world = 1): also the ADAM step with learning rate eta, fused into the loss
 * kernel — results of the three calls with grad_scale 1.  The batch arrays
 * of _grad_sampled_dev are left in the handle's mz_replay_sample buffers.
 * _train_dev on the one-launch FC path (PER off) also draws step + 1's batch
 * into a second batch set, which the next call uses only while the shard
 * (games stored), the step, B and every other sampling call since still
 * match — identical results, the sampler off the next step's critical path
 * (env MZ_NO_BATCH_PREFETCH=1 turns it off).  Replaces, per step,
 * the learner's fetch of the buffer + get_batch + learning! iteration
 * (Learning.jl:329-404).                                                    */
int mz_learner_grad_sampled_dev(mz_handle* h, int32_t B, uint32_t step, float* grad_dev,
                                float* losses_dev, void* stream);
int mz_learner_train_dev(mz_handle* h, int32_t B, uint32_t step, double eta, float* losses_dev,
                         void* stream);

/* L consecutive learner iterations (Learning.jl:327-404) at steps step0 ..
 * step0+L-1, eta[i] the learning rate of step step0+i (host array): the
 * results of L mz_learner_train_dev calls, bit for bit.  In ref_semantics
 * (Q11) the update θ_{s+1} = ADAM(θ_s, 2θ_s) does not read the data, and with
 * PER off step s's batch is keyed by s, so the engine runs the ADAM
 * iterations of many steps in one launch and their unrolls + losses side by
 * side (L·B workgroups instead of B).  losses_dev:
 * NULL or [L][8] (per step the six losses of mz_learner_train_dev);
 * theta_dev: NULL or [L][nflat], the flat parameters (Flux order, the
 * mz_weights_get layout of all three nets back to back) after each step.
 * 1 <= L <= 256.  FC: chain launches (mz_learn_chain: the ADAM iterations,
 * each step's θ scattered into its own image in a bank, Σθ² per step, the
 * batches) of up to 32 steps, each followed by unroll launches
 * (mz_learn_multi*) of up to 16 steps side by side; ResNet: the same chain
 * launches feeding the mz_runroll_* launches with the steps on gridDim.z
 * (rlearner_multi).  The corrected mode and PER run the L steps one after
 * another.  Replaces L iterations of the learner loop.                      */
int mz_learner_train_multi_dev(mz_handle* h, int32_t B, uint32_t step0, int32_t L, const double* eta,
                               float* losses_dev, float* theta_dev, void* stream);

/* PER (conf.PER, ReplayBuffer.jl:133-145, 168-183; Learning.jl:400-404).
 * With PER the shard keeps per-position priorities (initialised by
 * save_game: |root_value − target_value|^PER_alpha, game priority = max),
 * get_batch samples games and positions by priority and fills
 * batch->weights, and the learner weights its losses.  The fused learner
 * calls (mz_learner_train_dev / _grad_sampled_dev) then update the sampled
 * positions' priorities from the unroll's values; after mz_replay_sample +
 * mz_learner_grad_dev call mz_replay_update_priorities (it uses the batch of
 * the last sample and the last unroll).  The reference's update_priorities!
 * cannot run (`minimum(a, b)`, a K+2-element slice); this is its intended
 * reading: positions pos..min(pos+K, len), samples in batch order.          */
int mz_replay_update_priorities(mz_handle* h, void* stream);
/* Debug/parity: priorities of game i of the shard (0 = oldest held), T of
 * them, and its game priority; synchronises.                                */
int mz_replay_get_priorities(mz_handle* h, int32_t i, float* priorities, float* game_priority);

/* Debug/parity: game i of the shard (0 = oldest held), buffers sized for
 * max_moves + 1 moves (layouts as mz_replay_save_game); any pointer may be
 * NULL.  And the slots' games in progress: moves recorded, boards (G, W*H*C)
 * as 0/1 bytes, player to move.  Both synchronise.                         */
int mz_replay_get_game(mz_handle* h, int32_t i, int32_t* T, uint8_t* obs, int32_t* actions,
                       float* rewards, int32_t* to_play, float* child_visits, float* root_values);
int mz_selfplay_slots(mz_handle* h, int32_t* history_len, uint8_t* board, int32_t* player);

/* ---- Actor–learner loop (self_play! ‖ learning!) -----
 * The reference runs self_play! (SelfPlay.jl:384-419) and learning!
 * (Learning.jl:306-438) as two processes coupled by RemoteChannels (quirk
 * Q16): self-play take!s the training step once per game, the learner put!s
 * it once per step, and every checkpoint_interval steps the learner queues
 * its nets on remote_NNs (capacity 1, starting with the initial nets) which
 * self-play then take!s — the actors run one checkpoint behind.  On the
 * device, for the G lockstep slots of mz_selfplay_init:
 *   mz_train_init: the actors' weight set and the queue start as copies of
 *     the engine's current (initial) nets; learner step t = 0; B = batch.
 *   mz_train_init_at: the same from learner step t0 (a resume: pass the
 *     training_step mz_checkpoint_load returned; the Cos η phase, the
 *     training_steps bound, the temperature and the checkpoint cadence then
 *     continue from t0).  Checkpoints hold the learner's nets and ADAM state,
 *     not the actors' or queued sets, so a resume restarts the one-checkpoint
 *     lag: actors and queue start as copies of the loaded learner nets.
 *   mz_train_run: `moves` times: one self-play move of every slot with the
 *     ACTORS' nets (mz_selfplay_move, move key move0 + m); each game plays
 *     at the temperature visit_softmax_temperature_fn(t) of the step t at
 *     which it started (play_game takes T once per game, SelfPlay.jl:396-407;
 *     games in progress at mz_train_init_at take that of t0); then one
 *     learner step per game saved by that move (mz_learner_train_dev with
 *     step t+1, eta = Cos(t+1)) while t <= training_steps; after step t with
 *     t % checkpoint_interval == 0 and t > 1 the actors take the queued nets
 *     and the learner's nets are queued, and — when a networks path is set and
 *     t > round(0.9 training_steps) — the learner's state is written to
 *     <networks_path>/<t>.safetensors (mz_checkpoint_save; Learning.jl:416-432).
 *     Deliberate deviation: the G games run in lockstep on one weight set, so
 *     a refresh reaches every slot at once, games in progress included; the
 *     reference's single actor takes new nets only between games
 *     (SelfPlay.jl:399-401).  Reads the shard's game counter back once per
 *     move (one kernel stores it into pinned host memory and the host spins
 *     on it, bounded; the stream's work up to that move is then complete).
 *     state_out[4] = {t, num_played_games, actor refreshes,
 *     learner steps of this call}; losses_dev (device, 6 floats, or NULL) =
 *     the last step's.  The learner steps of one move run as one
 *     mz_learner_train_multi_dev chunk across the refresh points (the chain
 *     launch copies out θ of the last two refresh steps for the actors' and
 *     queued sets, and writes the actors' search images; with a networks path
 *     the chunks end at each refresh).
 *     Data parallel (after mz_dp_init, world > 1): the move's finished-game
 *     count is summed over the ranks (RCCL) and every rank takes that many
 *     learner steps on its own shard, so the ref_semantics replicas stay
 *     bit-identical.
 *   mz_train_move / mz_train_learn: the two halves of one mz_train_run move,
 *     for a host that exchanges the count itself (torch.distributed, a Julia
 *     Distributed host): mz_train_move plays one move and returns the games it
 *     saved on this rank (*nfin); mz_train_learn takes `steps` learner steps
 *     (capped at training_steps) with the refreshes, state_out as above.
 *   mz_train_set_networks_path: conf.networks_path (Constructors.jl:47) for
 *     the periodic checkpoints; NULL or "" (the default) writes none.
 *   mz_train_weights_get: the learner's, actors' or queued nets (Flux order).
 * oracle/mz_oracle.c ora_train_loop restates it.                            */
enum { MZ_TRAIN_LEARNER = 0, MZ_TRAIN_ACTOR = 1, MZ_TRAIN_QUEUED = 2 };
int mz_train_init(mz_handle* h, int32_t batch_size);
int mz_train_init_at(mz_handle* h, int32_t batch_size, int64_t t0);
int mz_train_set_networks_path(mz_handle* h, const char* networks_path);
int mz_train_run(mz_handle* h, int32_t moves, uint32_t move0, uint32_t game_offset, int64_t* state_out,
                 float* losses_dev, void* stream);
int mz_train_move(mz_handle* h, uint32_t move, uint32_t game_offset, int64_t* nfin, void* stream);
int mz_train_learn(mz_handle* h, int64_t steps, float* losses_dev, int64_t* state_out, void* stream);
int mz_train_weights_get(mz_handle* h, int which, int net, float* flat, size_t n);

/* ---- Checkpoints -------------------------------------------
 * Replace serialize(joinpath(networks_path, "$(step)_<net>.bin"), net)
 * (Learning.jl:424-431) and play.jl's deserialize: one safetensors file with
 * the three nets' Flux.params arrays ("<net>.<i>", Julia column-major bytes,
 * shape = the Julia shape reversed), the ADAM moments and βp state, and
 * metadata (training_step, network kind, config).  Load checks every shape
 * against this engine and restores weights + optimiser state (resume).      */
int mz_checkpoint_save(mz_handle* h, const char* path, int64_t training_step);
int mz_checkpoint_load(mz_handle* h, const char* path, int64_t* training_step);

/* Name of the search kernel variant the last search launched (for profiles):
 * mz_search_small{1,2,4} (T games per workgroup, G <= 4 x #CUs) or the
 * 16-game MFMA tile kernel mz_search_kernel_{lds,hbm}[_res].  Environment
 * MZ_SEARCH_KERNEL=tile16|small (read at create) forces a family.          */
const char* mz_search_variant(const mz_handle* h);

/* The learner unroll's kernels of the last ResNet learner step, "+"-joined
 * (e.g. mz_runroll_chain_r+mz_runroll_pred_n1), for profiles; "none" before. */
const char* mz_learner_variant(const mz_handle* h);

/* Wait for the engine's work (the device, or the pair mz_set_sync_stream
 * named) and report a device fault.  A kernel that gives up waiting for a
 * cross-workgroup publish (a bounded poll, 2 s) sets a fault word instead of
 * hanging; this and every host-synchronous call then fail once with the
 * message.  What it invalidates: the outputs of the launches since the last
 * synchronisation — search results, the games self-play stored from them in
 * the replay shard, losses and read-outs.  The ref_semantics weights and
 * ADAM state stay valid (their update does not read those outputs, Q11);
 * after a fault re-create the shard (mz_selfplay_init) before training on it. */
int mz_sync(mz_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* MZ_H */
