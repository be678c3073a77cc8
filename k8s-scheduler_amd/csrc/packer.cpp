// packer.cpp -- host-side packing of Kubernetes-shaped inputs into the engine's SoA arrays, with
// Go-exact quantity parsing.  Reference: anchor/predicate.go:10-105.
//
// Go semantics reproduced here (amd64, Go >= 1.13 strconv):
//   strconv.ParseInt(s, 10, 64): [+-]digits, no underscores, overflow is an error.
//   strconv.ParseFloat(s, 32):  decimal or 0x-hex ('p' exponent required) literals, Go-style
//                               underscores, inf/infinity/nan words; value = nearest float32;
//                               overflow -> error (ErrRange), underflow -> 0 / subnormal, no error.
//   int64(float64):             truncation, 0x8000000000000000 when out of range or NaN (CVTTSD2SQ).
//   int64 + - *:                two's-complement wrap.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>

#include "ksched.h"

namespace {

inline int64_t wrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t wrap_sub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
inline char lo(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }
inline bool is_dig(char c) { return c >= '0' && c <= '9'; }
inline bool is_hex(char c) { return is_dig(c) || (lo(c) >= 'a' && lo(c) <= 'f'); }

bool parse_int64(std::string_view s, int64_t *out) {
    if (s.empty()) return false;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; s.remove_prefix(1); }
    if (s.empty()) return false;
    uint64_t v = 0;
    for (char c : s) {
        if (!is_dig(c)) return false;
        uint64_t d = (uint64_t)(c - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX;
    if (v > lim) return false;
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

// strconv underscoreOK: '_' only between digits (a base prefix counts as a digit).
bool underscores_ok(std::string_view s) {
    if (!s.empty() && (s[0] == '+' || s[0] == '-')) s.remove_prefix(1);
    char saw = '^';
    size_t i = 0;
    bool hex = false;
    if (s.size() >= 2 && s[0] == '0' && (lo(s[1]) == 'b' || lo(s[1]) == 'o' || lo(s[1]) == 'x')) {
        i = 2; saw = '0'; hex = lo(s[1]) == 'x';
    }
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if (is_dig(c) || (hex && is_hex(c))) { saw = '0'; continue; }
        if (c == '_') { if (saw != '0') return false; saw = '_'; continue; }
        if (saw == '_') return false;
        saw = '!';
    }
    return saw != '_';
}

size_t common_prefix_ci(std::string_view s, const char *word) {
    size_t k = 0;
    while (word[k] && k < s.size() && lo(s[k]) == word[k]) ++k;
    return k;
}

enum class FloatErr { ok, syntax, range };

// ParseFloat(s, 32) -> value widened to double.
FloatErr parse_float32(std::string_view s, double *out) {
    if (s.empty()) return FloatErr::syntax;
    {   // special words (atof.go special())
        size_t j = 0;
        double sign = 1.0;
        if (s[0] == '+' || s[0] == '-') { sign = s[0] == '-' ? -1.0 : 1.0; j = 1; }
        if (j < s.size() && lo(s[j]) == 'i') {
            size_t k = common_prefix_ci(s.substr(j), "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) {
                if (j + k != s.size()) return FloatErr::syntax;
                *out = sign * HUGE_VAL;
                return FloatErr::ok;
            }
        } else if (j == 0 && lo(s[0]) == 'n' && common_prefix_ci(s, "nan") == 3) {
            if (s.size() != 3) return FloatErr::syntax;
            *out = std::nan("");
            return FloatErr::ok;
        }
    }
    size_t i = 0;
    bool hex = false, digits = false, dot = false, unders = false;
    if (s[i] == '+' || s[i] == '-') ++i;
    if (i + 2 < s.size() && s[i] == '0' && lo(s[i + 1]) == 'x') { hex = true; i += 2; }
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '_') { unders = true; continue; }
        if (c == '.') { if (dot) break; dot = true; continue; }
        if (is_dig(c) || (hex && is_hex(c))) { digits = true; continue; }
        break;
    }
    if (!digits) return FloatErr::syntax;
    if (i < s.size() && lo(s[i]) == (hex ? 'p' : 'e')) {
        ++i;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
        if (i >= s.size() || !is_dig(s[i])) return FloatErr::syntax;
        for (; i < s.size() && (is_dig(s[i]) || s[i] == '_'); ++i)
            if (s[i] == '_') unders = true;
    } else if (hex) {
        return FloatErr::syntax;
    }
    if (i != s.size()) return FloatErr::syntax;
    if (unders && !underscores_ok(s)) return FloatErr::syntax;
    std::string buf;
    buf.reserve(s.size());
    for (char c : s) if (c != '_') buf.push_back(c);
    errno = 0;
    char *end = nullptr;
    const float f = std::strtof(buf.c_str(), &end);
    if (*end != '\0') return FloatErr::syntax;
    if (errno == ERANGE && std::isinf(f)) return FloatErr::range;
    *out = (double)f;
    return FloatErr::ok;
}

int64_t f64_to_i64_amd64(double x) {
    if (std::isnan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

bool ends_with(std::string_view s, std::string_view suf) {
    return s.size() >= suf.size() && s.substr(s.size() - suf.size()) == suf;
}

}  // namespace

extern "C" int ksched_parse_cpu(const char *s, int64_t *out) {
    if (!out) return KSCHED_E_INVALID;
    *out = 0;
    if (!s) return KSCHED_OK;
    std::string_view v(s);
    if (ends_with(v, "m")) {  // milli-cores: ParseInt or errFatal (anchor/predicate.go:12-16)
        int64_t x;
        if (!parse_int64(v.substr(0, v.size() - 1), &x)) return KSCHED_E_PARSE;
        *out = x;
        return KSCHED_OK;
    }
    double c;
    if (parse_float32(v, &c) == FloatErr::ok) *out = f64_to_i64_amd64(c * 1000.0);  // :18-20
    return KSCHED_OK;  // ParseFloat error -> 0 (:23)
}

extern "C" int ksched_parse_memory(const char *s, int64_t *out) {
    if (!out) return KSCHED_E_INVALID;
    *out = 0;
    if (!s) return KSCHED_OK;
    std::string_view v(s);
    int64_t x;
    if (ends_with(v, "Ki")) {  // anchor/predicate.go:28-33
        if (!parse_int64(v.substr(0, v.size() - 2), &x)) return KSCHED_E_PARSE;
        *out = x;
    } else if (ends_with(v, "Mi")) {  // :36-41, m * 1024 wraps like Go
        if (!parse_int64(v.substr(0, v.size() - 2), &x)) return KSCHED_E_PARSE;
        *out = (int64_t)((uint64_t)x * 1024u);
    }
    return KSCHED_OK;  // any other suffix ("Gi", bytes, "G") -> 0 (:43)
}

extern "C" int ksched_parse_pods(const char *s, int64_t *out) {
    if (!out) return KSCHED_E_INVALID;
    *out = 0;
    if (!s) return KSCHED_OK;
    int64_t x;
    if (!parse_int64(s, &x)) return KSCHED_E_PARSE;  // anchor/predicate.go:48-50
    *out = x;
    return KSCHED_OK;
}

// Node price annotation (README.md:43-48 lists "0.80", "0.05", ...).  The reference has no price
// code; the build parses the annotation as a float32 decimal and rejects non-finite values.
extern "C" int ksched_parse_price(const char *s, float *out) {
    if (!out || !s) return KSCHED_E_INVALID;
    double v;
    if (parse_float32(s, &v) != FloatErr::ok || !std::isfinite(v)) return KSCHED_E_PARSE;
    // "-0" and "0" are the same price: canonical +0 keeps the lowest-index tie rule intact where
    // keys are ranked by bit pattern (the merge's order-preserving key codes)
    *out = v == 0.0 ? 0.0f : (float)v;
    return KSCHED_OK;
}

extern "C" int ksched_pack_nodes(int64_t n, const char *const *names, const char *const *cap_cpu,
                                 const char *const *cap_mem, const char *const *cap_pods, int64_t nb,
                                 const char *const *bound_node, const int64_t *cont_off,
                                 const char *const *cont_cpu, const char *const *cont_mem,
                                 int64_t *alloc_cpu, int64_t *alloc_mem, int64_t *alloc_pods) {
    if (n < 0 || nb < 0 || !alloc_cpu || !alloc_mem || !alloc_pods) return KSCHED_E_INVALID;
    if (n > 0 && (!names || !cap_cpu || !cap_mem || !cap_pods)) return KSCHED_E_INVALID;
    if (nb > 0 && (!bound_node || !cont_off)) return KSCHED_E_INVALID;
    std::unordered_map<std::string_view, int64_t> index;
    index.reserve((size_t)n * 2);
    for (int64_t i = 0; i < n; ++i) {
        // capacity, not allocatable (anchor/predicate.go:58-60)
        int r;
        if ((r = ksched_parse_cpu(cap_cpu[i], &alloc_cpu[i])) != KSCHED_OK) return r;
        if ((r = ksched_parse_memory(cap_mem[i], &alloc_mem[i])) != KSCHED_OK) return r;
        if ((r = ksched_parse_pods(cap_pods[i], &alloc_pods[i])) != KSCHED_OK) return r;
        index.emplace(names[i] ? std::string_view(names[i]) : std::string_view(), i);
    }
    // usedResource (anchor/predicate.go:83-105): unbound pods are skipped; each bound pod adds its
    // containers' cpu/mem and ONE pod.
    for (int64_t b = 0; b < nb; ++b) {
        if (!bound_node[b] || bound_node[b][0] == '\0') continue;
        auto it = index.find(std::string_view(bound_node[b]));
        if (it == index.end()) return KSCHED_E_UNKNOWN_NODE;
        const int64_t j = it->second;
        int64_t uc = 0, um = 0;
        for (int64_t c = cont_off[b]; c < cont_off[b + 1]; ++c) {
            int64_t v;
            int r;
            if ((r = ksched_parse_cpu(cont_cpu ? cont_cpu[c] : nullptr, &v)) != KSCHED_OK) return r;
            uc = wrap_add(uc, v);
            if ((r = ksched_parse_memory(cont_mem ? cont_mem[c] : nullptr, &v)) != KSCHED_OK) return r;
            um = wrap_add(um, v);
        }
        alloc_cpu[j] = wrap_sub(alloc_cpu[j], uc);
        alloc_mem[j] = wrap_sub(alloc_mem[j], um);
        alloc_pods[j] = wrap_sub(alloc_pods[j], 1);
    }
    return KSCHED_OK;
}

extern "C" int ksched_pack_pods(int64_t p, const int64_t *cont_off, const char *const *cont_cpu,
                                const char *const *cont_mem, int64_t *req_cpu, int64_t *req_mem,
                                int64_t *req_pods) {
    if (p < 0 || (p > 0 && (!cont_off || !req_cpu || !req_mem || !req_pods))) return KSCHED_E_INVALID;
    for (int64_t i = 0; i < p; ++i) {  // requestedResource, anchor/predicate.go:69-81
        int64_t rc = 0, rm = 0, rp = 0;
        for (int64_t c = cont_off[i]; c < cont_off[i + 1]; ++c) {
            int64_t v;
            int r;
            if ((r = ksched_parse_cpu(cont_cpu ? cont_cpu[c] : nullptr, &v)) != KSCHED_OK) return r;
            rc = wrap_add(rc, v);
            if ((r = ksched_parse_memory(cont_mem ? cont_mem[c] : nullptr, &v)) != KSCHED_OK) return r;
            rm = wrap_add(rm, v);
            rp = wrap_add(rp, 1);  // one pod per CONTAINER in the request (:78)
        }
        req_cpu[i] = rc; req_mem[i] = rm; req_pods[i] = rp;
    }
    return KSCHED_OK;
}
