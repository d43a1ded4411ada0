// mz_selfplay_params.h — device self-play and the device
// replay shard (§8f-2): parameters shared by the host (mz_engine.hip) and the
// kernels (mz_selfplay.hip).
//
// Per game slot g (G slots played in lockstep, SelfPlay.jl:330-382):
//   env      board[g][osz] (0/1 bytes: planes [p1, p2, empty], col-major cells),
//            player[g] (1 or 2), over[g]; the synthetic Atari-like env
//            (frames = 4): board[g] = the current 84x84 frame, ekey[g] its key;
//   history  GameHistory (Constructors.jl:6-16) of the game in progress, up to
//            T = max_moves + 1 moves: obs[g][T][osz] bytes (one frame per move
//            when frames > 0: the observation stacks the last `frames`), act / rew / tp /
//            rv [g][T], cv [g][T][A], len[g] = moves recorded.
// Replay shard (ReplayBuffer.jl:133-161, PER = false): a FIFO ring of `cap`
// finished games with the same per-game layout; game number n (1-based, the
// Dict key of save_game) lives in ring slot (n - 1) mod cap.
#pragma once
#include <stdint.h>

struct SpHist {                 // a set of game records: [n][T] ...
    uint8_t* obs;               // [n][T][osz]
    int32_t* act;               // [n][T] 1-based actions
    float* rew;                 // [n][T]
    int32_t* tp;                // [n][T] to_play before the move
    float* cv;                  // [n][T][A] child visit distributions
    float* rv;                  // [n][T] root values
    int32_t* len;               // [n] moves
    float* prio;                // [n][T] PER position priorities (ring only, conf.PER)
    float* gprio;               // [n] PER game priority = max(prio) (ring only)
};

struct SpParams {
    int G, env, W, H, osz, P, A, F, stacked, T, max_moves;
    int frames;                 // > 0: the env stacks its last `frames` frames (atari_synth), 0: board games
    uint8_t* board; int32_t* player; uint8_t* over;
    uint32_t* ekey;             // [G] synthetic Atari-like env state
    uint32_t reset_step;        // mz_sp_reset: the step key of the initial games
    SpHist hist;                // [G] games in progress
    SpHist ring;                // [cap] replay shard
    int cap;
    long long* counters;        // [0] num_played_games, [1] num_played_steps, [2] total_samples
    // search io (device buffers of the engine)
    float* obs; uint8_t* legal; int32_t* tp; const float* cv; const float* rv; const int32_t* act;
    int32_t* done;              // [G] finished this move
    int32_t* ring_pos;          // [G] ring slot of the finished game
    // evaluation play (competitive_play!, SelfPlay.jl:421-435): finished games
    // are tallied, not saved; with opponent = MZ_OPP_RANDOM the moves of the
    // player != muzero_player are uniform legal actions (select_opponent_action
    // :311-325) from the Philox OPPONENT stream keyed (game id, move step)
    int eval, opponent, muzero_player;
    uint32_t step, game_offset;
    uint64_t seed;
    long long* eval_counts;     // [4] games, muzero wins, opponent wins, draws
    // PER (conf.PER): initial priorities of a stored game (save_game, ReplayBuffer.jl:133-145)
    int per, per_alpha, td;
    const float* disc_pow;
    // temperature_threshold (SelfPlay.jl:344-346): a game with >= temp_threshold
    // moves recorded plays at temperature 0 (-1 = nothing: every slot at `temperature`)
    float temperature; int temp_threshold; float* temp_g;   // temp_g [G]
    // actor-learner loop (mz_train_run): each game keeps the temperature of its first move,
    // as play_game(env, temperature, ...) takes it once per game (SelfPlay.jl:396-407);
    // tgame [G] holds it (nullptr: every move uses `temperature`)
    float* tgame;
};

// get_batch + make_target (ReplayBuffer.jl:5-50, 73-107, 188-217) on the shard
struct RpSampleParams {
    int B, K, A, osz, P, F, stacked, T, td, cap;
    int frames;                 // the env's frame stack (0: stacked observations, Q15)
    uint64_t seed; uint32_t step;
    SpHist ring;
    const long long* counters;
    const float* disc_pow;      // [td + 2]: f32(discount^n) as Julia's Float32^Int
    float* obs; float* actions; float* tv; float* tr; float* tpol; float* gscale;
    int32_t* index;             // [B][2]: (game number, position) — index_batch
    // PER (conf.PER): sample_n_games / sample_position by priority (:73-107)
    // from the cumulative game probabilities of mz_rp_per_prep; raw IS weights
    // 1/(total_samples·p_game·p_pos), normalised by mz_rp_per_norm (:211-215)
    int per;
    const float* per_cum;       // [n held] cumulative f32 game probabilities (oldest first)
    const float* per_p;         // [n held] game probabilities
    const long long* per_total; // total_samples of the held games
    float* weights;             // [B]
};
