# LibMZ.jl — the Julia binding of libmz (include/mz.h) a MuZero.jl maintainer
# adds to the reference (deveshjawla/MuZero.jl), next to src/SelfPlay.jl and
# src/Learning.jl.  Every `ccall` matches include/mz.h: Cint status (0 = OK),
# 1-based actions, column-major arrays in the reference's own shapes, so Julia
# arrays pass with no transpose.  The executable mirror of this file is
# muzero.jl_amd/abi.py (ctypes); this image has no Julia toolchain, so the file
# is reviewed, not run (INTEGRATION.md).
module LibMZ

using Flux: params, relu, tanh

const libmz = get(ENV, "LIBMZ", joinpath(@__DIR__, "..", "muzero.jl_amd", "lib", "libmz.so"))

# ---- PODs: field order and types exactly as include/mz.h --------------------
struct MzConfig                         # Config, src/Constructors.jl:18-52
    seed::Int32; observation_shape::NTuple{3,Int32}; action_space_size::Int32; players::Int32
    stacked_observations::Int32; muzero_player::Int32; intermediate_rewards::Int32
    num_workers::Int32; selfplay_on_gpu::Int32; max_moves::Int32; temperature_threshold::Int32
    dirichlet_alpha::Float32; exploration_eps::Float32; pb_c_base::Int32; pb_c_init::Float32
    discount::Float32; num_iters::Int32; replay_buffer_size::Int32; num_unroll_steps::Int32
    td_steps::Int32; PER::Int32; PER_alpha::Int32; training_steps::Int32; batch_size::Int32
    checkpoint_interval::Int32; value_loss_weight::Float32
end
struct MzFFHP                           # FeedForwardHP, src/Constructors.jl:62-75
    width_hidden::Int32; depth_representation::Int32; depth_prediction::Int32; depth_dynamics::Int32
    depth_policy::Int32; depth_value::Int32; depth_reward::Int32; depth_state_head::Int32
    use_batch_norm::Int32; batch_norm_momentum::Float32; hidden_state_size::Int32; reward_activation::Int32
end
struct MzResNetHP                       # ResNetHP, src/Constructors.jl:77-90 (+ the fields its heads read, Q12)
    num_blocks::Int32; num_filters::Int32; conv_kernel_size::NTuple{2,Int32}
    num_second_head_filters::Int32; num_first_head_filters::Int32; batch_norm_momentum::Float32
    downsample::Int32; depth_policy::Int32; depth_value::Int32; width_hidden::Int32; reward_activation::Int32
end
struct MzBatch                          # the tuple of get_batch, src/ReplayBuffer.jl:216
    batch_size::Int32
    observation::Ptr{Float32}; actions::Ptr{Float32}; target_values::Ptr{Float32}
    target_rewards::Ptr{Float32}; target_policies::Ptr{Float32}; gradient_scale::Ptr{Float32}
    weights::Ptr{Float32}               # weight_batch (:211-215); C_NULL without PER
end

const NET_REPR, NET_PRED, NET_DYN = Cint(0), Cint(1), Cint(2)
const ACT_IDENTITY, ACT_RELU, ACT_TANH = Int32(0), Int32(1), Int32(2)
const ENV_TICTACTOE, ENV_CONNECT4, ENV_ATARI = Cint(0), Cint(1), Cint(2)   # ENV_ATARI: the synthetic frame-stacked env of configs[4]
const SP_TRAIN, SP_EVAL, OPP_SELF, OPP_RANDOM = Cint(0), Cint(1), Cint(0), Cint(1)
const LEARN_REF_SEMANTICS, LEARN_CORRECTED = Cint(0), Cint(1)
const TRAIN_LEARNER, TRAIN_ACTOR, TRAIN_QUEUED = Cint(0), Cint(1), Cint(2)

act_code(f) = f === tanh ? ACT_TANH : f === relu ? ACT_RELU : ACT_IDENTITY

MzConfig(c) = MzConfig(c.seed, Int32.(c.observation_shape), length(c.action_space), length(c.players),
    c.stacked_observations, c.muzero_player, c.intermediate_rewards, c.num_workers, c.selfplay_on_gpu,
    c.max_moves, something(c.temperature_threshold, -1), c.dirichlet_α, c.exploration_ϵ, c.pb_c_base,
    c.pb_c_init, c.discount, c.num_iters, c.replay_buffer_size, c.num_unroll_steps, c.td_steps, c.PER,
    c.PER_alpha, c.training_steps, c.batch_size, c.checkpoint_interval, c.value_loss_weight)
MzFFHP(h) = MzFFHP(h.width_hidden, h.depth_representation, h.depth_prediction, h.depth_dynamics,
    h.depth_policy, h.depth_value, h.depth_reward, h.depth_state_head, h.use_batch_norm,
    h.batch_norm_momentum, h.hidden_state_size, act_code(h.reward_activation))
# ResNetHP declares neither width_hidden nor reward_activation although its heads read them (Q12)
MzResNetHP(h; width_hidden=64, reward_activation=tanh) = MzResNetHP(h.num_blocks, h.num_filters,
    Int32.(h.conv_kernel_size), h.num_second_head_filters, h.num_first_head_filters, h.batch_norm_momentum,
    h.downsample, h.depth_policy, h.depth_value, width_hidden, act_code(reward_activation))

mutable struct Engine
    h::Ptr{Cvoid}
end

last_error(e::Engine) = unsafe_string(ccall((:mz_last_error, libmz), Cstring, (Ptr{Cvoid},), e.h))
check(e::Engine, rc) = rc == 0 || error("libmz: ", last_error(e))

"""Engine(conf, hyper; device, max_games, rng_seed) — replaces init_representation /
init_prediction / init_dynamics (src/Learning.jl:87-142, 148-255) and the process
setup of games/tictactoe/main.jl:15-28.  One engine per GPU."""
function Engine(conf, hyper; device=0, max_games=512, rng_seed=UInt64(1234))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    rc = if hasproperty(hyper, :num_filters)            # ResNetHP
        ccall((:mz_engine_create_resnet, libmz), Cint,
              (Ref{MzConfig}, Ref{MzResNetHP}, Cint, Cint, UInt64, Ref{Ptr{Cvoid}}),
              MzConfig(conf), MzResNetHP(hyper), device, max_games, rng_seed, out)
    else
        ccall((:mz_engine_create, libmz), Cint,
              (Ref{MzConfig}, Ref{MzFFHP}, Cint, Cint, UInt64, Ref{Ptr{Cvoid}}),
              MzConfig(conf), MzFFHP(hyper), device, max_games, rng_seed, out)
    end
    rc == 0 || error("libmz: ", unsafe_string(ccall((:mz_create_error, libmz), Cstring, ())))
    e = Engine(out[])
    finalizer(x -> ccall((:mz_engine_destroy, libmz), Cvoid, (Ptr{Cvoid},), x.h), e)
    return e
end

# ---- weights: vcat(vec.(Flux.params(net))...) (Dense: W (out,in) column-major, then b)
function set_weights!(e::Engine, net::Cint, chain)
    flat = reduce(vcat, vec.(collect(params(chain))))
    check(e, ccall((:mz_weights_set, libmz), Cint, (Ptr{Cvoid}, Cint, Ptr{Float32}, Csize_t),
                   e.h, net, flat, length(flat)))
end
function get_weights(e::Engine, net::Cint)
    n = Ref{Csize_t}(0)
    check(e, ccall((:mz_net_param_count, libmz), Cint, (Ptr{Cvoid}, Cint, Ref{Csize_t}), e.h, net, n))
    flat = Vector{Float32}(undef, n[])
    check(e, ccall((:mz_weights_get, libmz), Cint, (Ptr{Cvoid}, Cint, Ptr{Float32}, Csize_t), e.h, net, flat, n[]))
    flat
end
set_nets!(e::Engine, NNs) = (set_weights!(e, NET_REPR, NNs.representation);
                             set_weights!(e, NET_PRED, NNs.prediction); set_weights!(e, NET_DYN, NNs.dynamics))

# the Chain call (src/Learning.jl:87-142): x (W,H,C,N) -> out0 (and out1 for PRED / DYN)
forward!(e::Engine, net::Cint, x::Array{Float32}, out0::Array{Float32}, out1=nothing) =
    check(e, ccall((:mz_net_forward, libmz), Cint,
                   (Ptr{Cvoid}, Cint, Ptr{Float32}, Cint, Ptr{Float32}, Ptr{Float32}),
                   e.h, net, x, size(x, ndims(x)), out0, out1 === nothing ? C_NULL : out1))

"""mcts_search!(e, obs (W,H,Cs,G), legal (A,G) UInt8, to_play (G)) — G × (run_mcts +
select_action + store_search_stats!), src/SelfPlay.jl:230-306, 115-122."""
function mcts_search!(e::Engine, obs::Array{Float32,4}, legal::Matrix{UInt8}, to_play::Vector{Int32};
                      exploration=true, rng_step::Integer, game_offset::Integer=0, temperature::Float32=1f0)
    G = size(obs, 4); A = size(legal, 1)
    child_visits = Matrix{Float32}(undef, A, G); root_value = Vector{Float32}(undef, G)
    action = Vector{Int32}(undef, G)
    check(e, ccall((:mz_mcts_search, libmz), Cint,
                   (Ptr{Cvoid}, Cint, Ptr{Float32}, Ptr{UInt8}, Ptr{Int32}, Cint, UInt32, UInt32, Float32,
                    Ptr{Float32}, Ptr{Float32}, Ptr{Int32}),
                   e.h, G, obs, legal, to_play, exploration, rng_step, game_offset, temperature,
                   child_visits, root_value, action))
    return child_visits, root_value, action
end

# ParameterSchedulers 0.2.3 Cos(λ0=1e-4, λ1=1e-1, period=10) under Stateful (src/Learning.jl:319, 382);
# the caller keeps the schedule (`next!(schedule)`) and passes eta
cos_eta(t) = abs(1e-4 - 1e-1) * (1 + cos(2π * (t - 1) / 10)) / 2 + min(1e-4, 1e-1)

"""learner_step!(e, batch, eta) — one learning! iteration (src/Learning.jl:327-413) on
batch = get_batch(buffer)[2]; eta = next!(schedule) (:382).  Returns the losses
(value, reward, policy, Σθ² of repr / pred / dyn)."""
function learner_step!(e::Engine, batch, eta::Real)
    obs, acts, tv, tr, tp, w, gs = batch
    acts32 = Float32.(acts)
    losses = Vector{Float32}(undef, 6)
    GC.@preserve obs acts32 tv tr tp w gs begin
        b = MzBatch(size(obs, 4), pointer(obs), pointer(acts32), pointer(tv), pointer(tr), pointer(tp),
                    pointer(gs), w === nothing ? C_NULL : pointer(w))
        check(e, ccall((:mz_learner_step, libmz), Cint, (Ptr{Cvoid}, Ref{MzBatch}, Float64, Ptr{Float32}),
                       e.h, b, Float64(eta), losses))
    end
    return losses
end

"""learner_mode!(e, LEARN_CORRECTED) — real backpropagation through the unroll
(FC nets with or without BatchNorm, ResNet nets with or without the downsampler) instead of the reference's
∇ = 2θ (quirk Q11)."""
learner_mode!(e::Engine, mode::Cint) =
    check(e, ccall((:mz_learner_set_mode, libmz), Cint, (Ptr{Cvoid}, Cint), e.h, mode))

# ---- device self-play and replay shard (play_game's loop body + ReplayBuffer.jl on the GPU)
selfplay_init!(e::Engine, env::Cint, G, replay_games) =
    check(e, ccall((:mz_selfplay_init, libmz), Cint, (Ptr{Cvoid}, Cint, Cint, Cint), e.h, env, G, replay_games))
selfplay_move!(e::Engine, step; offset=0, temperature=1f0) =
    check(e, ccall((:mz_selfplay_move, libmz), Cint, (Ptr{Cvoid}, UInt32, UInt32, Float32, Ptr{Cvoid}),
                   e.h, step, offset, temperature, C_NULL))
selfplay_mode!(e::Engine, mode::Cint; opponent=OPP_SELF, mzp=1) =
    check(e, ccall((:mz_selfplay_mode, libmz), Cint, (Ptr{Cvoid}, Cint, Cint, Cint), e.h, mode, opponent, mzp))
function eval_results(e::Engine)               # competitive_play!: (games, MuZero wins, opponent wins, draws)
    r = zeros(Int64, 4)
    check(e, ccall((:mz_eval_results, libmz), Cint, (Ptr{Cvoid}, Ptr{Int64}), e.h, r))
    Tuple(r)
end
function replay_counts(e::Engine)              # (num_played_games, num_played_steps, total_samples), held
    c = zeros(Int64, 3); held = Ref{Int32}(0)
    check(e, ccall((:mz_replay_counts, libmz), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ref{Int32}), e.h, c, held))
    Tuple(c), held[]
end
learner_train!(e::Engine, B, step, eta; losses=C_NULL) =  # get_batch + learning! on the device shard
    check(e, ccall((:mz_learner_train_dev, libmz), Cint, (Ptr{Cvoid}, Int32, UInt32, Float64, Ptr{Float32}, Ptr{Cvoid}),
                   e.h, B, step, eta, losses, C_NULL))
# length(etas) consecutive learning! iterations from step0 (ref_semantics, Q11: the ADAM chain in one
# launch, the unrolls side by side in a second); losses: C_NULL or a device [8, L] buffer
learner_train_multi!(e::Engine, B, step0, etas::Vector{Float64}; losses=C_NULL) =
    check(e, ccall((:mz_learner_train_multi_dev, libmz), Cint,
                   (Ptr{Cvoid}, Int32, UInt32, Int32, Ptr{Float64}, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                   e.h, B, step0, length(etas), etas, losses, C_NULL, C_NULL))

"""The actor–learner loop of self_play! ‖ learning! (src/SelfPlay.jl:384-419,
src/Learning.jl:306-438; quirk Q16) on one GPU: `moves` self-play moves with the
actors' nets, one learner step per finished game, the actors one checkpoint behind.
Returns (learner step t, games played, actor refreshes, steps of this call)."""
train_init!(e::Engine, B) = check(e, ccall((:mz_train_init, libmz), Cint, (Ptr{Cvoid}, Int32), e.h, B))
function train_run!(e::Engine, moves; move0=0, offset=0)
    st = zeros(Int64, 4)
    check(e, ccall((:mz_train_run, libmz), Cint, (Ptr{Cvoid}, Int32, UInt32, UInt32, Ptr{Int64}, Ptr{Float32}, Ptr{Cvoid}),
                   e.h, moves, move0, offset, st, C_NULL, C_NULL))
    Tuple(st)
end
# the two halves of one train_run! move, for a Distributed.jl host that sums `nfin` over the workers itself:
# every worker then takes the global count of learner steps (the replicas stay identical, SURVEY §8e)
function train_move!(e::Engine, move; offset=0)
    n = zeros(Int64, 1)
    check(e, ccall((:mz_train_move, libmz), Cint, (Ptr{Cvoid}, UInt32, UInt32, Ptr{Int64}, Ptr{Cvoid}),
                   e.h, move, offset, n, C_NULL))
    n[1]
end
function train_learn!(e::Engine, steps)
    st = zeros(Int64, 4)
    check(e, ccall((:mz_train_learn, libmz), Cint, (Ptr{Cvoid}, Int64, Ptr{Float32}, Ptr{Int64}, Ptr{Cvoid}),
                   e.h, steps, C_NULL, st, C_NULL))
    Tuple(st)
end
function train_weights(e::Engine, which::Cint, net::Cint)
    flat = similar(get_weights(e, net))
    check(e, ccall((:mz_train_weights_get, libmz), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Float32}, Csize_t),
                   e.h, which, net, flat, length(flat)))
    flat
end

# host-synchronous calls wait only for `stream` (a HIP stream handle) and the engine's own; narrow=false: all work
set_sync_stream!(e::Engine, stream::Ptr{Cvoid}; narrow=true) =
    check(e, ccall((:mz_set_sync_stream, libmz), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cint), e.h, stream, Cint(narrow)))

# ---- data-parallel learner over RCCL without torch (one engine per GPU / Distributed.jl worker)
function dp_unique_id()                        # on rank 0; send the 128 bytes to the other workers
    id = zeros(UInt8, 128)
    ccall((:mz_dp_unique_id, libmz), Cint, (Ptr{UInt8},), id) == 0 || error("mz_dp_unique_id")
    id
end
dp_init!(e::Engine, rank, world, id) =
    check(e, ccall((:mz_dp_init, libmz), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}), e.h, rank, world, id))
learner_train_dp!(e::Engine, B, step, eta; losses=C_NULL) =   # data term, RCCL all-reduce, ADAM(1/world, + 2θ)
    check(e, ccall((:mz_learner_train_dp, libmz), Cint, (Ptr{Cvoid}, Int32, UInt32, Float64, Ptr{Float32}, Ptr{Cvoid}),
                   e.h, B, step, eta, losses, C_NULL))

# ---- checkpoints (the safetensors file replacing serialize(...), src/Learning.jl:424-431)
checkpoint_save(e::Engine, path, step) =
    check(e, ccall((:mz_checkpoint_save, libmz), Cint, (Ptr{Cvoid}, Cstring, Int64), e.h, path, step))
function checkpoint_load!(e::Engine, path)
    step = Ref{Int64}(0)
    check(e, ccall((:mz_checkpoint_load, libmz), Cint, (Ptr{Cvoid}, Cstring, Ref{Int64}), e.h, path, step))
    step[]
end

end # module
