"""Learner driver — host mirror of learning! (src/Learning.jl:306-438).

Each step: get_batch from the (per-GPU) replay buffer, then one
ref_semantics learner step on the GPU (mz_learner_step: K-step unroll,
losses, gradient 2θ per quirk Q11, Flux ADAM with the Cos(λ0=1e-4,
λ1=1e-1, period=10) learning rate, Learning.jl:318-319,382).  Data-parallel
training splits the step: the gradient's data term -> RCCL
all-reduce (sum) of the flat bucket -> ADAM on data·(1/world) + 2θ, so every
replica applies the same update, equal to the single-GPU one in ref_semantics
at any world size.
"""
import numpy as np

from .config import cos_schedule
from .networks import NET_DYN, NET_PRED, NET_REPR


class Learner:
    def __init__(self, engine, buffer, process_group=None):
        self.eng = engine
        self.buffer = buffer
        self.conf = engine.conf
        self.training_step = 0
        self.losses = None
        self.pg = process_group

    def step(self):
        """One iteration of Learning.jl:327-413 (single GPU)."""
        _, batch = self.buffer.get_batch(self.training_step)
        eta = cos_schedule(self.training_step + 1)              # next!(schedule), :382
        l = self.eng.learner_step(batch, eta)
        self.training_step += 1
        # the three reported losses (:385-393) differ only in their L2 term
        data = float(l[0]) + float(l[1]) + float(l[2])
        self.losses = dict(representation=data + float(l[3]), prediction=data + float(l[4]),
                           dynamics=data + float(l[5]), value=float(l[0]), policy=float(l[2]))
        return self.losses

    def nets(self):
        return [self.eng.get_weights(n) for n in (NET_REPR, NET_PRED, NET_DYN)]


def allreduce_step(engine, dev_batch_ptrs, B, grad, losses, step, world, all_reduce, stream=None):
    """Data-parallel learner step on device buffers: the DATA TERM of the
    gradient into `grad` (a device tensor of engine.grad_count() floats; zero
    in ref_semantics, where only Σθ² depends on θ, Q11), `all_reduce(grad)`
    (sum over ranks; RCCL via torch.distributed on GPU, gloo in CPU tests),
    then ADAM on ∇ = Σ·(1/world) + 2θ.  The rank-invariant 2θ is added after
    the exchange (mz_adam_kernel), so every replica's update equals the
    single-GPU update bit for bit at EVERY world size in ref_semantics — an
    exchange of the full 2θ would not: a sequential f32 sum of eight equal
    terms differs from 8x for ~44 % of inputs (dp_gradient)."""
    engine.learner_grad_dev(dev_batch_ptrs, B, grad.data_ptr(), losses.data_ptr(), stream=stream)
    if world > 1:
        all_reduce(grad)
    engine.learner_apply_dev(grad.data_ptr(), 1.0 / world, cos_schedule(step + 1), stream=stream)


def dp_gradient(data_grad, theta, world, all_reduce):
    """Host reference of the data-parallel gradient mz_adam_kernel applies:
    ∇ = (Σ_ranks data_grad) · f32(1/world) + 2θ, in f32 with the device's
    operation order (the data term's product rounded, then the sum).
    data_grad is summed in place by all_reduce (world > 1)."""
    if world > 1:
        all_reduce(data_grad)
    d = np.asarray(data_grad, dtype=np.float32) * np.float32(1.0 / world)
    return (d + np.asarray(theta, dtype=np.float32) * np.float32(2)).astype(np.float32)
