// mz_checkpoint.cpp — checkpoints: mz_checkpoint_save / _load.
//
// Replaces `serialize(joinpath(networks_path, "$(step)_<net>.bin"), net)`
// (Learning.jl:424-431) and its `deserialize` in play.jl:12-14: Julia's
// serializer is unreadable outside Julia, so one checkpoint is one
// safetensors file (an 8-byte little-endian header length, a JSON header,
// raw little-endian data), readable from Julia (SafeTensors.jl), Python
// (safetensors, numpy) and C, and loadable without executing anything.
//
// Tensors:
//   "<net>.<i>"       the i-th array of Flux.params(<net>), <net> in
//                     representation / prediction / dynamics; its bytes are
//                     the Julia array's column-major bytes and its shape is
//                     the Julia shape reversed (the row-major view of the
//                     same bytes), e.g. a Dense W (out, in) is stored [in, out];
//   "adam.m", "adam.v"  the ADAM moments over the three nets back to back
//                     (F32, the engine's flat order = the nets' Flux order);
//   "adam.beta_pow"   (β1^t, β2^t) (F64), the optimiser's βp state.
// __metadata__: format, network ("fc" | "resnet"), training_step, config
// (JSON).  Loading checks every parameter's shape against this engine.
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "mz_ckpt_iface.h"
#include "mz_st_header.h"

namespace {

std::string esc(const std::string& s) {
    std::string o;
    for (char c : s) {
        if (c == '"' || c == '\\') o += '\\';
        o += c;
    }
    return o;
}

struct Entry {
    std::string name, dtype;
    std::vector<int64_t> shape;   // safetensors (row-major) shape
    const void* data;
    size_t bytes;
};

}  // namespace

extern "C" {

int mz_checkpoint_save(mz_handle* h, const char* path, int64_t training_step) {
    if (!h) return -2;
    if (!path) return mz_set_error(h, "null path");
    const size_t n = mz_flat_count(h);
    std::vector<float> flat(n), m(n), v(n);
    double bp[2];
    if (mz_state_get(h, flat.data(), m.data(), v.data(), bp)) return -1;
    std::vector<Entry> ents;
    for (const MzParamDesc& d : mz_param_table(h)) {
        std::vector<int64_t> shp(d.jshape.rbegin(), d.jshape.rend());
        ents.push_back(Entry{d.name, "F32", shp, flat.data() + d.off, d.count * 4});
    }
    ents.push_back(Entry{"adam.m", "F32", {(int64_t)n}, m.data(), n * 4});
    ents.push_back(Entry{"adam.v", "F32", {(int64_t)n}, v.data(), n * 4});
    ents.push_back(Entry{"adam.beta_pow", "F64", {2}, bp, 16});
    std::string hdr = "{\"__metadata__\":{\"format\":\"libmz-checkpoint-1\",\"network\":\"" + mz_net_kind(h) +
                      "\",\"training_step\":\"" + std::to_string((long long)training_step) + "\",\"config\":\"" +
                      esc(mz_describe(h)) + "\"}";
    size_t off = 0;
    for (const Entry& e : ents) {
        hdr += ",\"" + e.name + "\":{\"dtype\":\"" + e.dtype + "\",\"shape\":[";
        for (size_t i = 0; i < e.shape.size(); ++i) hdr += (i ? "," : "") + std::to_string((long long)e.shape[i]);
        hdr += "],\"data_offsets\":[" + std::to_string(off) + "," + std::to_string(off + e.bytes) + "]}";
        off += e.bytes;
    }
    hdr += "}";
    while (hdr.size() % 8) hdr += ' ';
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return mz_set_error(h, std::string("cannot write ") + tmp);
    const uint64_t hl = hdr.size();
    bool ok = std::fwrite(&hl, 8, 1, f) == 1 && std::fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size();
    for (const Entry& e : ents) ok = ok && std::fwrite(e.data, 1, e.bytes, f) == e.bytes;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        return mz_set_error(h, std::string("writing ") + path + " failed");
    }
    return 0;
}

int mz_checkpoint_load(mz_handle* h, const char* path, int64_t* training_step) {
    if (!h) return -2;
    if (!path) return mz_set_error(h, "null path");
    FILE* f = std::fopen(path, "rb");
    if (!f) return mz_set_error(h, std::string("cannot open ") + path);
    std::unique_ptr<FILE, int (*)(FILE*)> guard(f, std::fclose);
    uint64_t hl = 0;
    if (std::fread(&hl, 8, 1, f) != 1 || hl > (1u << 28)) return mz_set_error(h, "not a safetensors file");
    std::string hdr(hl, '\0');
    if (std::fread(&hdr[0], 1, hl, f) != hl) return mz_set_error(h, "truncated header");
    mzst::JV root;
    const std::string perr = mzst::parse_header(hdr.data(), hdr.size(), &root);
    if (!perr.empty()) return mz_set_error(h, perr);
    std::fseek(f, 0, SEEK_END);
    const long long fsize = std::ftell(f);
    auto read = [&](const std::string& name, const char* dtype, size_t esz, std::vector<int64_t> shape,
                    void* dst) -> int {
        long long off = 0;
        const std::string err = mzst::entry_span(root, name, dtype, esz, shape, hl, fsize, &off);
        if (!err.empty()) return mz_set_error(h, err);
        size_t cnt = 1;
        for (int64_t d : shape) cnt *= (size_t)d;
        std::fseek(f, (long)off, SEEK_SET);
        if (std::fread(dst, 1, cnt * esz, f) != cnt * esz) return mz_set_error(h, name + ": short read");
        return 0;
    };
    const size_t n = mz_flat_count(h);
    std::vector<float> flat(n), m(n), v(n);
    double bp[2];
    for (const MzParamDesc& d : mz_param_table(h)) {
        std::vector<int64_t> shp(d.jshape.rbegin(), d.jshape.rend());
        if (int rc = read(d.name, "F32", 4, shp, flat.data() + d.off)) return rc;
    }
    if (int rc = read("adam.m", "F32", 4, {(int64_t)n}, m.data())) return rc;
    if (int rc = read("adam.v", "F32", 4, {(int64_t)n}, v.data())) return rc;
    if (int rc = read("adam.beta_pow", "F64", 8, {2}, bp)) return rc;
    if (training_step) {
        *training_step = 0;
        auto md = root.obj.find("__metadata__");
        if (md != root.obj.end() && md->second.t == mzst::JV::OBJ) {
            auto ts = md->second.obj.find("training_step");
            if (ts != md->second.obj.end() && ts->second.t == mzst::JV::STR) *training_step = std::strtoll(ts->second.str.c_str(), nullptr, 10);
        }
    }
    return mz_state_set(h, flat.data(), m.data(), v.data(), bp);
}

}  // extern "C"
