// mz_st_header.h — the safetensors header reader of mz_checkpoint_load
// (SURVEY §8f-3), host C++ only and free of the engine, so the same code is
// compiled into libmz and into the CPU AddressSanitizer harness
// (tests/sanitize/ckpt_header_asan.cpp).
//
// A safetensors file is an 8-byte little-endian header length n, n bytes of
// JSON, then the data.  The header is untrusted input: the reader bounds the
// JSON nesting depth, never reads outside [p, e) (every look-ahead is checked
// against the end; numbers are parsed from a bounded copy), and an entry's
// data span must satisfy 0 <= begin <= end and 8 + n + end <= file size.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace mzst {

struct JV {
    enum T { NUL, NUM, STR, ARR, OBJ, BOOL } t = NUL;
    double num = 0;
    std::string str;
    std::vector<JV> arr;
    std::map<std::string, JV> obj;
};

constexpr int kMaxDepth = 32;          // nesting of objects / arrays (a checkpoint header uses 3)

struct JP {
    const char* p;
    const char* e;
    bool ok = true;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
    bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
    bool lit(const char* w) {          // a literal keyword, bounds-checked
        const size_t n = std::strlen(w);
        if ((size_t)(e - p) < n || std::memcmp(p, w, n) != 0) return false;
        p += n;
        return true;
    }
    std::string string() {
        std::string s;
        if (!eat('"')) { ok = false; return s; }
        while (p < e && *p != '"') {
            if (*p == '\\') {
                if (e - p < 2) { ok = false; return s; }
                ++p;
                const char c = *p++;
                if (c == 'n') s += '\n';
                else if (c == 't') s += '\t';
                else if (c == 'u') {               // \uXXXX: kept as '?' (names and dtypes are ASCII)
                    if (e - p < 4) { ok = false; return s; }
                    s += '?';
                    p += 4;
                } else s += c;
            } else {
                s += *p++;
            }
        }
        if (p >= e) { ok = false; return s; }
        ++p;
        return s;
    }
    JV value(int depth = 0) {
        JV v;
        ws();
        if (p >= e || depth > kMaxDepth) { ok = false; return v; }
        if (*p == '{') {
            ++p;
            v.t = JV::OBJ;
            if (eat('}')) return v;
            do {
                std::string k = string();
                if (!ok || !eat(':')) { ok = false; return v; }
                v.obj[k] = value(depth + 1);
            } while (ok && eat(','));
            if (!ok || !eat('}')) ok = false;
        } else if (*p == '[') {
            ++p;
            v.t = JV::ARR;
            if (eat(']')) return v;
            do v.arr.push_back(value(depth + 1)); while (ok && eat(','));
            if (!ok || !eat(']')) ok = false;
        } else if (*p == '"') {
            v.t = JV::STR;
            v.str = string();
        } else if (lit("null")) {
        } else if (lit("true")) {
            v.t = JV::BOOL; v.num = 1;
        } else if (lit("false")) {
            v.t = JV::BOOL;
        } else {                               // a number: strtod on a NUL-terminated copy
            char buf[64];
            size_t n = 0;
            while (p + n < e && n < sizeof(buf) - 1 && std::strchr("+-.0123456789eE", p[n]) && p[n]) ++n;
            std::memcpy(buf, p, n);
            buf[n] = '\0';
            char* q = nullptr;
            v.t = JV::NUM;
            v.num = std::strtod(buf, &q);
            if (n == 0 || q != buf + n) { ok = false; return v; }
            p += n;
        }
        return v;
    }
};

// Parse header bytes [h, h + n) into *root (an object); "" or the reason.
inline std::string parse_header(const char* h, size_t n, JV* root) {
    JP jp{h, h + n};
    *root = jp.value();
    jp.ws();
    if (!jp.ok || root->t != JV::OBJ) return "bad safetensors header";
    if (jp.p != jp.e) return "trailing bytes after the safetensors header";
    return "";
}

// Validate entry `name` (dtype, shape, element size esz) against the file:
// header length hl, file size fsize.  On success *off = the data's absolute
// file offset.  "" or the reason.
inline std::string entry_span(const JV& root, const std::string& name, const char* dtype, size_t esz,
                              const std::vector<int64_t>& shape, uint64_t hl, long long fsize, long long* off) {
    auto it = root.obj.find(name);
    if (it == root.obj.end() || it->second.t != JV::OBJ) return "checkpoint lacks " + name;
    const JV& e = it->second;
    auto dt = e.obj.find("dtype");
    auto sh = e.obj.find("shape");
    auto of = e.obj.find("data_offsets");
    if (dt == e.obj.end() || sh == e.obj.end() || of == e.obj.end() || dt->second.t != JV::STR ||
        sh->second.t != JV::ARR || of->second.t != JV::ARR || of->second.arr.size() != 2 ||
        of->second.arr[0].t != JV::NUM || of->second.arr[1].t != JV::NUM)
        return "bad header entry " + name;
    if (dt->second.str != dtype) return name + ": dtype " + dt->second.str + ", expected " + dtype;
    std::vector<int64_t> got;
    for (const JV& x : sh->second.arr) {
        if (x.t != JV::NUM || !(x.num >= 0 && x.num < 9.0e15) || x.num != (double)(int64_t)x.num)
            return name + ": bad shape";
        got.push_back((int64_t)x.num);
    }
    if (got != shape) return name + ": shape differs from this engine's network";
    size_t cnt = 1;
    for (int64_t d : shape) cnt *= (size_t)d;
    const double a = of->second.arr[0].num, b = of->second.arr[1].num;
    if (!(a >= 0 && b >= a && b < 9.0e15) || a != (double)(long long)a || b != (double)(long long)b)
        return name + ": bad data offsets";
    const long long base = 8 + (long long)hl;
    if ((long long)b - (long long)a != (long long)(cnt * esz) || base + (long long)b > fsize)
        return name + ": bad data offsets";
    *off = base + (long long)a;
    return "";
}

}  // namespace mzst
