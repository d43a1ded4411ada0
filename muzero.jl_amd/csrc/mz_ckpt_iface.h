// mz_ckpt_iface.h — the engine's internal interface for checkpoints
// (mz_checkpoint.cpp).  Host-side only, not part of the C ABI.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/mz.h"

// One Flux parameter array: its name "<net>.<i>" (i = position in
// Flux.params of that net), its Julia (column-major) shape and its place in
// the engine's flat parameter vector.
struct MzParamDesc {
    std::string name;
    std::vector<int64_t> jshape;
    size_t off, count;
};

std::vector<MzParamDesc> mz_param_table(const mz_handle* h);
size_t mz_flat_count(const mz_handle* h);
// host copies of the whole training state: parameters (Flux order, three
// nets back to back), ADAM moments, βp = (β1^t, β2^t) (Learning.jl:385-397)
int mz_state_get(mz_handle* h, float* flat, float* m, float* v, double* beta_pow);
int mz_state_set(mz_handle* h, const float* flat, const float* m, const float* v, const double* beta_pow);
// "fc" | "resnet" and a JSON object describing config + hyper-parameters
std::string mz_net_kind(const mz_handle* h);
std::string mz_describe(const mz_handle* h);
int mz_set_error(mz_handle* h, const std::string& msg);
