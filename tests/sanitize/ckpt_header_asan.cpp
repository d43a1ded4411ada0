// CPU AddressSanitizer / UBSan harness of the checkpoint header reader
// (muzero.jl_amd/csrc/mz_st_header.h, the code mz_checkpoint_load runs; SURVEY
// §5 "sanitizer build of the host C/C++").  Every header is parsed from a heap
// buffer of exactly its length (no NUL after it), so a read past the end is an
// ASan report.  Cases: a valid checkpoint-shaped header, the malformed
// headers a hostile or truncated file can hold (deep nesting, negative or
// reversed offsets, spans past the file, truncated strings / escapes /
// literals / numbers), then random truncations and byte mutations of the
// valid one.  Exit 0 = every case handled, a sanitizer report aborts.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../muzero.jl_amd/csrc/mz_st_header.h"

static int failures = 0;

static bool parse_exact(const std::string& h, mzst::JV* root) {
    std::vector<char> buf(h.begin(), h.end());            // exactly h.size() bytes
    char* p = buf.empty() ? nullptr : buf.data();
    static char dummy;
    return mzst::parse_header(p ? p : &dummy, buf.size(), root).empty();
}

static void expect(bool cond, const char* what) {
    if (!cond) {
        std::fprintf(stderr, "FAIL: %s\n", what);
        ++failures;
    }
}

static std::string entry(const char* name, const char* dt, const char* shape, long long a, long long b) {
    return std::string("\"") + name + "\":{\"dtype\":\"" + dt + "\",\"shape\":" + shape +
           ",\"data_offsets\":[" + std::to_string(a) + "," + std::to_string(b) + "]}";
}

int main() {
    const std::string valid = "{\"__metadata__\":{\"format\":\"libmz-checkpoint-1\",\"training_step\":\"12\"}," +
                              entry("representation.0", "F32", "[27,64]", 0, 6912) + "," +
                              entry("adam.beta_pow", "F64", "[2]", 6912, 6928) + "}   ";
    const uint64_t hl = valid.size();
    const long long fsize = 8 + (long long)hl + 6928;
    mzst::JV root;
    expect(parse_exact(valid, &root), "valid header parses");
    long long off = -1;
    expect(mzst::entry_span(root, "representation.0", "F32", 4, {27, 64}, hl, fsize, &off).empty() &&
               off == 8 + (long long)hl, "valid entry span");
    expect(mzst::entry_span(root, "adam.beta_pow", "F64", 8, {2}, hl, fsize, &off).empty(), "valid f64 entry");
    expect(!mzst::entry_span(root, "adam.beta_pow", "F64", 8, {2}, hl, fsize - 1, &off).empty(), "span past EOF");
    expect(!mzst::entry_span(root, "representation.0", "F32", 4, {64, 27}, hl, fsize, &off).empty(), "shape");
    expect(!mzst::entry_span(root, "representation.0", "F64", 8, {27, 64}, hl, fsize, &off).empty(), "dtype");
    expect(!mzst::entry_span(root, "missing", "F32", 4, {1}, hl, fsize, &off).empty(), "missing entry");

    // offsets: negative begin, reversed, non-numeric, fractional huge
    const char* bad_offsets[] = {"[-4,6908]", "[6912,0]", "[\"0\",6912]", "[0]", "[0,6912,1]", "[1e300,1e300]",
                                 "[0,1e300]", "[-1e300,6912]"};
    for (const char* o : bad_offsets) {
        std::string h = "{\"x\":{\"dtype\":\"F32\",\"shape\":[27,64],\"data_offsets\":" + std::string(o) + "}}";
        mzst::JV r;
        if (parse_exact(h, &r))
            expect(!mzst::entry_span(r, "x", "F32", 4, {27, 64}, h.size(), 1 << 20, &off).empty(), o);
    }
    // shapes that are not counts
    const char* bad_shapes[] = {"[-27,64]", "[27.5,64]", "[\"27\",64]", "27", "[1e300,1]", "[null,64]"};
    for (const char* sh : bad_shapes) {
        std::string h = "{\"x\":{\"dtype\":\"F32\",\"shape\":" + std::string(sh) + ",\"data_offsets\":[0,6912]}}";
        mzst::JV r;
        if (parse_exact(h, &r))
            expect(!mzst::entry_span(r, "x", "F32", 4, {27, 64}, h.size(), 1 << 20, &off).empty(), sh);
    }
    // malformed JSON: every one must be rejected without reading past the buffer
    const char* bad_json[] = {"", "{", "}", "{\"a\"", "{\"a\":", "{\"a\":1,", "{\"a\\", "{\"a\\u12",
                              "{\"a\":\"x\\", "{\"a\":nul", "{\"a\":tru", "{\"a\":1e", "{\"a\":-", "{\"a\":[1,2",
                              "{\"a\":{\"b\":[}}", "{\"a\":1}x", "[1,2]", "\"s\"", "{\"a\" 1}", "{1:2}",
                              "{\"a\":1 \"b\":2}", "{\"a\":+}", "{\"a\":.}"};
    for (const char* j : bad_json) {
        mzst::JV r;
        expect(!parse_exact(j, &r), j);
    }
    // nesting far past the bound: rejected, no stack exhaustion
    for (int depth : {mzst::kMaxDepth + 2, 1000, 200000}) {
        std::string h = "{\"a\":" + std::string(depth, '[') + std::string(depth, ']') + "}";
        mzst::JV r;
        expect(!parse_exact(h, &r), "deep nesting");
    }
    {
        std::string h = "{\"a\":" + std::string(8, '[') + std::string(8, ']') + "}";   // shallow: fine
        mzst::JV r;
        expect(parse_exact(h, &r), "shallow nesting");
    }
    // every truncation of the valid header, then random byte mutations
    for (size_t n = 0; n < valid.size(); ++n) {
        mzst::JV r;
        if (parse_exact(valid.substr(0, n), &r))
            for (const char* name : {"representation.0", "adam.beta_pow"})
                (void)mzst::entry_span(r, name, "F32", 4, {27, 64}, n, fsize, &off);
    }
    std::mt19937 rng(1234);
    const char alphabet[] = "{}[]\":,\\u0123456789-+.eEtrufalsn \x01\xff";
    int parsed = 0;
    for (int it = 0; it < 200000; ++it) {
        std::string h = valid;
        const int edits = 1 + (int)(rng() % 4);
        for (int k = 0; k < edits; ++k) {
            const size_t pos = rng() % h.size();
            switch (rng() % 3) {
                case 0: h[pos] = alphabet[rng() % (sizeof(alphabet) - 1)]; break;
                case 1: h.erase(pos, 1 + rng() % 8); break;
                default: h.insert(pos, 1, alphabet[rng() % (sizeof(alphabet) - 1)]); break;
            }
            if (h.empty()) break;
        }
        mzst::JV r;
        if (parse_exact(h, &r)) {
            ++parsed;
            for (const char* name : {"representation.0", "adam.beta_pow", "__metadata__"})
                (void)mzst::entry_span(r, name, "F32", 4, {27, 64}, h.size(), fsize, &off);
        }
    }
    std::printf("ckpt_header_asan: %d failures, %d of 200000 mutations parsed\n", failures, parsed);
    return failures ? 1 : 0;
}
