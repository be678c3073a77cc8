/*
 * oracle/cpu_ref.c -- CPU restatement of the yinwoods/k8s-scheduler scheduling hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (k8s-scheduler_amd/) never links,
 * imports or calls anything here, and has no CPU fallback.
 *
 * Parity status: the reference is Go with no go.mod and no tests and no
 * Go toolchain exists in this image, so the reference cannot be run.  This restatement is pinned
 * only by (a) the README demo known-answer test (best-price -> node "pxee", README.md:43-58) and
 * (b) the hand-derived example values of SURVEY.md section 8c, both held in tests/golden/.  For the
 * resource-score path it is otherwise "parity unpinned" (Oracle).
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp (no -march=native), see oracle/Makefile.
 * Every IEEE double operation below is written in the reference's evaluation order, with no FMA
 * contraction -- the Go amd64 (GOAMD64=v1) compiler never fuses.
 *
 * Reference anchors (paths relative to /root/reference):
 *   parseCpu            anchor/predicate.go:10-24
 *   parseMemory         anchor/predicate.go:26-44
 *   parsePod            anchor/predicate.go:46-53
 *   allocatableResource anchor/predicate.go:56-67
 *   requestedResource   anchor/predicate.go:69-81
 *   usedResource        anchor/predicate.go:83-105
 *   predicate (fit)     anchor/predicate.go:127-150
 *   fractionOfCapacity  anchor/scores.go:3-8
 *   getBalancedResourceScore anchor/scores.go:10-18
 *   getLeastRequestedScore   anchor/scores.go:20-25
 *   balancedResourceScore    anchor/priorities.go:5-15
 *   leastRequestedScore      anchor/priorities.go:17-23
 *   priorities (score loop + argmax) anchor/priorities.go:25-62
 *   schedulePod / schedulePods       anchor/schedule.go:68-89, 185-197
 */
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_OK 0
#define OR_E_PARSE (-3)
#define OR_E_INVALID (-1)
#define OR_NO_FIT (-1)
#define OR_NO_POSITIVE_SCORE (-2)

enum { OR_PRIORITY_RESOURCE = 0, OR_PRIORITY_BEST_PRICE = 1 };
enum { OR_DOMAIN_ALL = 0, OR_DOMAIN_FEASIBLE = 1 };

typedef struct or_opts {
    int32_t priority;   /* OR_PRIORITY_* */
    int32_t domain;     /* OR_DOMAIN_*   (best-price always ranges over feasible nodes) */
    int32_t use_labels; /* build-defined label-bitset predicate */
    int32_t pad;
} or_opts;

/* ------------------------------------------------------------------------------------------ */
/* Go strconv emulation                                                                        */
/* ------------------------------------------------------------------------------------------ */

/* strconv.ParseInt(s, 10, 64): optional sign, decimal digits only (no underscores with base 10),
 * error on empty input or overflow.  Returns 0 or -1. */
static int go_parse_int64(const char *s, size_t n, int64_t *out)
{
    size_t i = 0;
    int neg = 0;
    uint64_t v = 0;
    if (n == 0) return -1;
    if (s[0] == '+' || s[0] == '-') { neg = (s[0] == '-'); i = 1; }
    if (i == n) return -1;
    for (; i < n; i++) {
        unsigned d;
        if (s[i] < '0' || s[i] > '9') return -1;
        d = (unsigned)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10u) return -1;
        v = v * 10u + d;
    }
    if (!neg && v > (uint64_t)INT64_MAX) return -1;
    if (neg && v > (uint64_t)INT64_MAX + 1u) return -1;
    *out = neg ? (int64_t)(0u - v) : (int64_t)v;
    return 0;
}

static int lower_c(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

/* strconv underscoreOK (atoi.go): underscores only between digits / after a base prefix. */
static int go_underscore_ok(const char *s, size_t n)
{
    char saw = '^';
    size_t i = 0;
    int hex = 0;
    if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
    if (n >= 2 && s[0] == '0' && (lower_c(s[1]) == 'b' || lower_c(s[1]) == 'o' || lower_c(s[1]) == 'x')) {
        i = 2; saw = '0'; hex = lower_c(s[1]) == 'x';
    }
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if ((c >= '0' && c <= '9') || (hex && lower_c(c) >= 'a' && lower_c(c) <= 'f')) { saw = '0'; continue; }
        if (c == '_') { if (saw != '0') return 0; saw = '_'; continue; }
        if (saw == '_') return 0;
        saw = '!';
    }
    return saw != '_';
}

static size_t prefix_ci(const char *s, size_t n, const char *pat)
{
    size_t k = 0;
    while (pat[k] && k < n && lower_c((unsigned char)s[k]) == pat[k]) k++;
    return k;
}

/* strconv.ParseFloat(s, 32): 0 = ok (value widened to double), -1 = syntax error, -2 = range error.
 * Special forms follow atof.go special(); the syntax follows readFloat(); rounding is to nearest
 * float32 (glibc strtof is correctly rounded, as is Go). */
static int go_parse_float32(const char *s, size_t n, double *out)
{
    size_t i = 0, k;
    int base16 = 0, sawdigits = 0, sawdot = 0, underscores = 0;
    char buf[512];
    size_t bn = 0;
    float f;
    char *end;
    if (n == 0) return -1;
    /* special(): [+-]inf | [+-]infinity | nan  (case-insensitive) */
    {
        size_t j = 0;
        double sign = 1.0;
        int c0 = (unsigned char)s[0];
        if (c0 == '+' || c0 == '-') { sign = (c0 == '-') ? -1.0 : 1.0; j = 1; }
        if (j < n && lower_c((unsigned char)s[j]) == 'i') {
            k = prefix_ci(s + j, n - j, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) {
                if (j + k != n) return -1;
                *out = sign * INFINITY;
                return 0;
            }
        } else if (j == 0 && lower_c(c0) == 'n') {
            if (prefix_ci(s, n, "nan") == 3) {
                if (n != 3) return -1;
                *out = NAN;
                return 0;
            }
        }
    }
    /* readFloat syntax */
    if (s[i] == '+' || s[i] == '-') i++;
    if (i + 2 < n && s[i] == '0' && lower_c((unsigned char)s[i + 1]) == 'x') { base16 = 1; i += 2; }
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if (c == '_') { underscores = 1; continue; }
        if (c == '.') { if (sawdot) break; sawdot = 1; continue; }
        if (c >= '0' && c <= '9') { sawdigits = 1; continue; }
        if (base16 && lower_c(c) >= 'a' && lower_c(c) <= 'f') { sawdigits = 1; continue; }
        break;
    }
    if (!sawdigits) return -1;
    if (i < n && lower_c((unsigned char)s[i]) == (base16 ? 'p' : 'e')) {
        i++;
        if (i >= n) return -1;
        if (s[i] == '+' || s[i] == '-') i++;
        if (i >= n || s[i] < '0' || s[i] > '9') return -1;
        for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++)
            if (s[i] == '_') underscores = 1;
    } else if (base16) {
        return -1; /* hexadecimal mantissa requires a 'p' exponent */
    }
    if (underscores && !go_underscore_ok(s, i)) return -1;
    if (i != n) return -1;
    for (k = 0; k < n; k++) {
        if (s[k] == '_') continue;
        if (bn + 1 >= sizeof(buf)) return -1; /* absurdly long literal: treat as syntax error */
        buf[bn++] = s[k];
    }
    buf[bn] = 0;
    errno = 0;
    f = strtof(buf, &end);
    if (*end != 0) return -1;
    if (errno == ERANGE && isinf(f)) return -2;
    *out = (double)f;
    return 0;
}

/* Go's int64(float64) on amd64 (CVTTSD2SQ): truncation, 0x8000000000000000 when out of range/NaN. */
static int64_t go_f64_to_i64(double x)
{
    if (isnan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}

static int has_suffix(const char *s, size_t n, const char *suf)
{
    size_t m = strlen(suf);
    return n >= m && memcmp(s + n - m, suf, m) == 0;
}

/* parseCpu, anchor/predicate.go:10-24.  s == NULL means the "cpu" key is absent. */
int or_parse_cpu(const char *s, int64_t *out)
{
    size_t n;
    double c;
    if (!s) { *out = 0; return OR_OK; }
    n = strlen(s);
    if (has_suffix(s, n, "m")) {
        int64_t v;
        if (go_parse_int64(s, n - 1, &v)) return OR_E_PARSE; /* errFatal, predicate.go:15 */
        *out = v;
        return OR_OK;
    }
    if (go_parse_float32(s, n, &c) == 0) { *out = go_f64_to_i64(c * 1000.0); return OR_OK; }
    *out = 0; /* ParseFloat error (syntax or range) -> 0, predicate.go:23 */
    return OR_OK;
}

/* parseMemory, anchor/predicate.go:26-44: "<int>Ki" -> n, "<int>Mi" -> n*1024 (wrapping), else 0. */
int or_parse_memory(const char *s, int64_t *out)
{
    size_t n;
    int64_t v;
    if (!s) { *out = 0; return OR_OK; }
    n = strlen(s);
    if (has_suffix(s, n, "Ki")) {
        if (go_parse_int64(s, n - 2, &v)) return OR_E_PARSE;
        *out = v;
        return OR_OK;
    }
    if (has_suffix(s, n, "Mi")) {
        if (go_parse_int64(s, n - 2, &v)) return OR_E_PARSE;
        *out = (int64_t)((uint64_t)v * 1024u);
        return OR_OK;
    }
    *out = 0;
    return OR_OK;
}

/* parsePod, anchor/predicate.go:46-53. */
int or_parse_pods(const char *s, int64_t *out)
{
    int64_t v;
    if (!s) { *out = 0; return OR_OK; }
    if (go_parse_int64(s, strlen(s), &v)) return OR_E_PARSE;
    *out = v;
    return OR_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Scores (IEEE double, reference operation order, no contraction)                             */
/* ------------------------------------------------------------------------------------------ */

static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

/* fractionOfCapacity, anchor/scores.go:3-8 */
static inline double fraction_of_capacity(int64_t req, int64_t cap)
{
    if (cap == 0) return 1.0;
    return (double)req / (double)cap;
}

/* getLeastRequestedScore, anchor/scores.go:20-25 */
static inline double least_requested(int64_t req, int64_t cap)
{
    if (cap == 0 || req > cap) return 0.0;
    return (double)wsub(cap, req) * 10.0 / (double)cap;
}

/* balancedResourceScore + getBalancedResourceScore, anchor/priorities.go:5-15, anchor/scores.go:10-18 */
static inline double balanced_resource(int64_t rc, int64_t rm, int64_t rp, int64_t ac, int64_t am, int64_t ap)
{
    double c = fraction_of_capacity(rc, ac);
    double m = fraction_of_capacity(rm, am);
    double p = fraction_of_capacity(rp, ap);
    double mean, cr, mr, pr, var;
    if (c >= 1.0 || m >= 1.0 || p >= 1.0) return 0.0;
    mean = ((c + m) + p) / 3.0;
    cr = (c - mean) * (c - mean);
    mr = (m - mean) * (m - mean);
    pr = (p - mean) * (p - mean);
    var = ((cr + mr) + pr) / 3.0;
    return (1.0 - var) * 10.0;
}

/* priorities score loop body, anchor/priorities.go:45-50: ((0 + balanced) + least) / 2 */
double or_score(int64_t rc, int64_t rm, int64_t rp, int64_t ac, int64_t am, int64_t ap)
{
    double b = balanced_resource(rc, rm, rp, ac, am, ap);
    double l = ((least_requested(rc, ac) + least_requested(rm, am)) + least_requested(rp, ap)) / 3.0;
    double s = 0.0;
    s += b;
    s += l;
    s /= 2.0;
    return s;
}

/* fit predicate, anchor/predicate.go:134-148, plus the build-defined label bitset (8a row 14) */
static inline int fits(int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                       int64_t ac, int64_t am, int64_t ap, uint64_t lab, int use_labels)
{
    if (ac < rc) return 0;
    if (am < rm) return 0;
    if (ap < rp) return 0;
    if (use_labels && (lab & sel) != sel) return 0;
    return 1;
}

/* Candidate key: larger is better; ties broken by lower node index (deterministic restatement of
 * the randomized map-order argmax at anchor/priorities.go:55-61).  For best-price the key is
 * -price among feasible nodes (README.md:37-64; build-defined). */
typedef struct { double key; int64_t idx; } cand_t;

static inline int cand_better(double ka, int64_t ia, double kb, int64_t ib)
{
    return ka > kb || (ka == kb && ia < ib);
}

/* Eligibility + key of one (pod, node) pair.  Returns 1 if the node may be selected. */
static inline int pair_key(const or_opts *o, int feas, int64_t rc, int64_t rm, int64_t rp,
                           int64_t ac, int64_t am, int64_t ap, float price, double *key)
{
    if (o->priority == OR_PRIORITY_BEST_PRICE) {
        if (!feas) return 0;
        *key = -(double)price;
        return 1;
    }
    if (o->domain == OR_DOMAIN_FEASIBLE && !feas) return 0;
    *key = or_score(rc, rm, rp, ac, am, ap);
    return *key > 0.0; /* strict '>' from maxScore = 0, priorities.go:55-61 */
}

static inline double out_score_of(const or_opts *o, double key)
{
    return o->priority == OR_PRIORITY_BEST_PRICE ? 0.0 - key : key; /* the price; both signed zeros give +0 */
}

/* ------------------------------------------------------------------------------------------ */
/* Sequential scheduler: schedulePods -> schedulePod -> predicate -> priorities -> bind          */
/* ------------------------------------------------------------------------------------------ */

/*
 * Schedules pods 0..p-1 in order against node state alloc_* (in/out; alloc = capacity - used,
 * anchor/predicate.go:56-67).  Per pod: feasible count over all nodes (predicate.go:127-150); if 0
 * -> NO_FIT (schedule.go:74-76, no commit); else the best node by key (priorities.go:45-61); if none
 * -> NO_POSITIVE_SCORE (the reference dereferences a nil node in bind, schedule.go:208: documented
 * divergence); else commit alloc[best] -= (req_cpu, req_mem, 1) -- used.Pod grows by ONE per bound
 * pod (predicate.go:102) even though the request counts one per container (predicate.go:78).
 * nthreads > 1 splits the node scan (OpenMP), with a deterministic combine.
 */
int or_schedule(const or_opts *o, int64_t n, int64_t *ac, int64_t *am, int64_t *ap,
                const uint64_t *labels, const float *price,
                int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                int32_t *out_idx, double *out_score, int32_t *out_feas, int nthreads)
{
    int64_t i;
    int use_labels = o->use_labels && labels && sel;
    if (n < 0 || p < 0) return OR_E_INVALID;
    if (o->priority == OR_PRIORITY_BEST_PRICE && !price) return OR_E_INVALID;
    if (nthreads < 1) nthreads = 1;
    for (i = 0; i < p; i++) {
        int64_t fc = 0, best = -1;
        double bkey = 0.0;
        const uint64_t s = use_labels ? sel[i] : 0;
#ifdef _OPENMP
        if (nthreads > 1) {
            int nt = nthreads, t;
            int64_t tfc[256];
            int64_t tbest[256];
            double tkey[256];
            if (nt > 256) nt = 256;
#pragma omp parallel num_threads(nt)
            {
                int tid = omp_get_thread_num();
                int ntt = omp_get_num_threads();
                int64_t lo = n * tid / ntt, hi = n * (tid + 1) / ntt, j;
                int64_t lfc = 0, lb = -1;
                double lk = 0.0;
                for (j = lo; j < hi; j++) {
                    double k;
                    int f = fits(rc[i], rm[i], rp[i], s, ac[j], am[j], ap[j], use_labels ? labels[j] : 0, use_labels);
                    lfc += f;
                    if (pair_key(o, f, rc[i], rm[i], rp[i], ac[j], am[j], ap[j], price ? price[j] : 0.f, &k)) {
                        if (lb < 0 || cand_better(k, j, lk, lb)) { lk = k; lb = j; }
                    }
                }
                tfc[tid] = lfc; tbest[tid] = lb; tkey[tid] = lk;
                if (tid == 0) nt = ntt;
            }
            for (t = 0; t < nt; t++) {
                fc += tfc[t];
                if (tbest[t] >= 0 && (best < 0 || cand_better(tkey[t], tbest[t], bkey, best))) { bkey = tkey[t]; best = tbest[t]; }
            }
        } else
#endif
        {
            int64_t j;
            for (j = 0; j < n; j++) {
                double k;
                int f = fits(rc[i], rm[i], rp[i], s, ac[j], am[j], ap[j], use_labels ? labels[j] : 0, use_labels);
                fc += f;
                if (pair_key(o, f, rc[i], rm[i], rp[i], ac[j], am[j], ap[j], price ? price[j] : 0.f, &k)) {
                    if (best < 0 || cand_better(k, j, bkey, best)) { bkey = k; best = j; }
                }
            }
        }
        out_feas[i] = (int32_t)fc;
        if (fc == 0) { out_idx[i] = OR_NO_FIT; out_score[i] = 0.0; continue; }
        if (best < 0) { out_idx[i] = OR_NO_POSITIVE_SCORE; out_score[i] = 0.0; continue; }
        out_idx[i] = (int32_t)best;
        out_score[i] = out_score_of(o, bkey);
        ac[best] = wsub(ac[best], rc[i]);
        am[best] = wsub(am[best], rm[i]);
        ap[best] = wsub(ap[best], 1);
    }
    return OR_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* FailedScheduling reasons: the failures list of predicate() (anchor/predicate.go:127-157)     */
/* ------------------------------------------------------------------------------------------ */

/* Per node, the FIRST failing check in the reference's order: CPU (predicate.go:134-138), Memory
 * (:139-143), Pod (:144-148); then the build-defined label check; 0 = the node is appended to the
 * feasible list (:149).  reason (n, may be NULL); counts[5] = nodes per code. */
int or_node_reasons(const or_opts *o, int64_t n, const int64_t *ac, const int64_t *am, const int64_t *ap,
                    const uint64_t *labels, int64_t rc, int64_t rm, int64_t rp, uint64_t sel,
                    uint8_t *reason, int64_t *counts)
{
    int64_t j;
    int k, use_labels = o->use_labels && labels;
    for (k = 0; k < 5; k++) counts[k] = 0;
    for (j = 0; j < n; j++) {
        int r;
        if (ac[j] < rc) r = 1;
        else if (am[j] < rm) r = 2;
        else if (ap[j] < rp) r = 3;
        else if (use_labels && (labels[j] & sel) != sel) r = 4;
        else r = 0;
        if (reason) reason[j] = (uint8_t)r;
        counts[r]++;
    }
    return OR_OK;
}

/* or_schedule with, for every pod, the reason counts of its predicate at its turn (counts: p*5).
 * The FailedScheduling event of a NO_FIT pod lists its nodes with codes 1..3 (predicate.go:157). */
int or_schedule_reasons(const or_opts *o, int64_t n, int64_t *ac, int64_t *am, int64_t *ap,
                        const uint64_t *labels, const float *price,
                        int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                        int32_t *out_idx, double *out_score, int32_t *out_feas, int64_t *counts)
{
    int64_t i;
    for (i = 0; i < p; i++) {
        int r;
        or_node_reasons(o, n, ac, am, ap, labels, rc[i], rm[i], rp[i], sel ? sel[i] : 0, NULL, counts + 5 * i);
        r = or_schedule(o, n, ac, am, ap, labels, price, 1, rc + i, rm + i, rp + i, sel ? sel + i : NULL,
                        out_idx + i, out_score + i, out_feas + i, 1);
        if (r != OR_OK) return r;
    }
    return OR_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Batched restatement: speculative top-K at a batch-start snapshot + ordered commit with the   */
/* touched-node re-score.  Must equal or_schedule bit-for-bit; it is the CPU model of the GPU   */
/* batched mode (Batched commit) and of its node-sharded multi-GPU form.             */
/* ------------------------------------------------------------------------------------------ */

/* One top-K entry as exchanged between shards: key, global node index and the node's state at
 * the snapshot (so a rank that does not own the node can re-score it after a commit). */
typedef struct or_rec {
    double key;
    int32_t idx;
    int32_t valid;
    int64_t a_cpu, a_mem, a_pods;
    uint64_t labels;
    float price;
    int32_t pad;
} or_rec; /* 56 bytes */

/* Local top-K of pods [0, nb) over nodes [0, n) of one shard (global index = offset + j), plus the
 * local feasible count.  recs: nb*K (sorted best first, invalid tail), fc: nb. */
int or_local_topk(const or_opts *o, int32_t K, int64_t offset, int64_t n,
                  const int64_t *ac, const int64_t *am, const int64_t *ap,
                  const uint64_t *labels, const float *price,
                  int64_t nb, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                  or_rec *recs, int64_t *fc)
{
    int64_t i, j;
    int use_labels = o->use_labels && labels && sel;
    for (i = 0; i < nb; i++) {
        or_rec *L = recs + i * K;
        int32_t cnt = 0, q;
        int64_t f = 0;
        const uint64_t s = use_labels ? sel[i] : 0;
        for (q = 0; q < K; q++) { memset(&L[q], 0, sizeof(or_rec)); L[q].idx = -1; }
        for (j = 0; j < n; j++) {
            double k;
            int ft = fits(rc[i], rm[i], rp[i], s, ac[j], am[j], ap[j], use_labels ? labels[j] : 0, use_labels);
            f += ft;
            if (!pair_key(o, ft, rc[i], rm[i], rp[i], ac[j], am[j], ap[j], price ? price[j] : 0.f, &k)) continue;
            if (cnt == K && !cand_better(k, offset + j, L[K - 1].key, L[K - 1].idx)) continue;
            /* insert, keeping (key desc, idx asc) order */
            q = cnt < K ? cnt : K - 1;
            while (q > 0 && cand_better(k, offset + j, L[q - 1].key, L[q - 1].idx)) { L[q] = L[q - 1]; q--; }
            L[q].key = k; L[q].idx = (int32_t)(offset + j); L[q].valid = 1;
            L[q].a_cpu = ac[j]; L[q].a_mem = am[j]; L[q].a_pods = ap[j];
            L[q].labels = labels ? labels[j] : 0; L[q].price = price ? price[j] : 0.f; L[q].pad = 0;
            if (cnt < K) cnt++;
        }
        fc[i] = f;
    }
    return OR_OK;
}

/* Merge R shard lists (recs_all[r][nb][K], fc_all[r][nb]) into one global list per pod. */
int or_merge_topk(int32_t K, int32_t R, int64_t nb, const or_rec *recs_all, const int64_t *fc_all,
                  or_rec *out, int64_t *fc_out)
{
    int64_t i;
    for (i = 0; i < nb; i++) {
        int32_t head[1024];
        int32_t q, r;
        int64_t f = 0;
        if (R > 1024) return OR_E_INVALID;
        for (r = 0; r < R; r++) { head[r] = 0; f += fc_all[(int64_t)r * nb + i]; }
        fc_out[i] = f;
        for (q = 0; q < K; q++) {
            int32_t br = -1;
            for (r = 0; r < R; r++) {
                const or_rec *h;
                if (head[r] >= K) continue;
                h = &recs_all[((int64_t)r * nb + i) * K + head[r]];
                if (!h->valid) continue;
                if (br < 0) { br = r; continue; }
                {
                    const or_rec *b = &recs_all[((int64_t)br * nb + i) * K + head[br]];
                    if (cand_better(h->key, h->idx, b->key, b->idx)) br = r;
                }
            }
            if (br < 0) { memset(&out[i * K + q], 0, sizeof(or_rec)); out[i * K + q].idx = -1; continue; }
            out[i * K + q] = recs_all[((int64_t)br * nb + i) * K + head[br]];
            head[br]++;
        }
    }
    return OR_OK;
}

typedef struct or_touched {
    int32_t idx;
    int32_t pad;
    int64_t s0[3];  /* state at the snapshot */
    int64_t cur[3]; /* current state */
    uint64_t labels;
    float price;
    int32_t pad2;
} or_touched;

/* The rescue of an exhausted list (the device's commit asks its merger workgroups for it, ksched_pipe.hip):
 * the node rows as the batch's score saw them -- the current state of every node the batch's touched set does
 * not hold -- so the best untouched node can be found by a full scan instead of truncating the batch. */
typedef struct or_rescue {
    int64_t n;
    const int64_t *ac, *am, *ap;
    const uint64_t *labels;
    const float *price;
    int64_t count;     /* rescues performed */
    int32_t shards;    /* the node rows as R contiguous shards (ksched.dist.shard_range): each shard's best
                          untouched node, then the best of the R (the device's node-sharded rescue); 1: one scan */
    int32_t max_per_batch;  /* rescues a batch may make before an exhausted list truncates it (< 0: no limit;
                               the device's KSCHED_RESCUE_MAX) */
    int32_t in_batch;  /* rescues made by the batch being committed */
} or_rescue;

/* The best node outside the touched set (touched[0, nt)) over rows [lo, hi) at their current state; -1: none
 * eligible.  anchor/priorities.go:45-61's loop, restricted to the untouched rows. */
static int64_t rescue_scan(const or_opts *o, const or_rescue *rs, int64_t lo, int64_t hi, int64_t rc, int64_t rm,
                           int64_t rp, uint64_t s, int ul, const or_touched *touched, int32_t nt, double *bk)
{
    int64_t j, bj = -1;
    int32_t t;
    for (j = lo; j < hi; j++) {
        double k;
        int ft, is_t = 0;
        for (t = 0; t < nt; t++) if (touched[t].idx == j) { is_t = 1; break; }
        if (is_t) continue;
        ft = fits(rc, rm, rp, s, rs->ac[j], rs->am[j], rs->ap[j], ul ? rs->labels[j] : 0, ul);
        if (!pair_key(o, ft, rc, rm, rp, rs->ac[j], rs->am[j], rs->ap[j], rs->price ? rs->price[j] : 0.f, &k))
            continue;
        if (bj < 0 || cand_better(k, j, *bk, bj)) { *bk = k; bj = j; }
    }
    return bj;
}

static int64_t commit_batch_impl(const or_opts *o, int32_t K, int64_t nb,
                                 const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                                 const or_rec *lists, const int64_t *fc0,
                                 or_touched *touched, int32_t *ntouched, int32_t max_touched,
                                 int32_t *out_idx, double *out_score, int32_t *out_feas, or_rescue *rs);

/* Ordered commit of a batch against merged lists.  Returns the number of pods resolved before the
 * first overflow (>= 1 when nb >= 1).  touched/ntouched carry the nodes committed in this batch.
 * The caller applies touched[].cur to its node state (owners only, when sharded). */
int64_t or_commit_batch(const or_opts *o, int32_t K, int64_t nb,
                        const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                        const or_rec *lists, const int64_t *fc0,
                        or_touched *touched, int32_t *ntouched, int32_t max_touched,
                        int32_t *out_idx, double *out_score, int32_t *out_feas)
{
    return commit_batch_impl(o, K, nb, rc, rm, rp, sel, lists, fc0, touched, ntouched, max_touched, out_idx,
                             out_score, out_feas, NULL);
}

static int64_t commit_batch_impl(const or_opts *o, int32_t K, int64_t nb,
                                 const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                                 const or_rec *lists, const int64_t *fc0,
                                 or_touched *touched, int32_t *ntouched, int32_t max_touched,
                                 int32_t *out_idx, double *out_score, int32_t *out_feas, or_rescue *rs)
{
    int64_t i;
    int use_labels = o->use_labels && sel;
    if (rs) rs->in_batch = 0;
    for (i = 0; i < nb; i++) {
        const or_rec *L = lists + i * K;
        const uint64_t s = use_labels ? sel[i] : 0;
        int64_t fc = fc0[i];
        int32_t t, q, cnt = 0, tb = -1, first_untouched = -1;
        double tkey = 0.0;
        int64_t w = -1, rj = -1;  /* rj: the rescued node (not in the list), when the rescue wins */
        double wkey = 0.0;
        for (t = 0; t < *ntouched; t++) {
            const or_touched *T = &touched[t];
            int f0 = fits(rc[i], rm[i], rp[i], s, T->s0[0], T->s0[1], T->s0[2], T->labels, use_labels);
            int f1 = fits(rc[i], rm[i], rp[i], s, T->cur[0], T->cur[1], T->cur[2], T->labels, use_labels);
            double k;
            fc += f1 - f0;
            if (pair_key(o, f1, rc[i], rm[i], rp[i], T->cur[0], T->cur[1], T->cur[2], T->price, &k)) {
                if (tb < 0 || cand_better(k, T->idx, tkey, touched[tb].idx)) { tkey = k; tb = t; }
            }
        }
        for (q = 0; q < K; q++) {
            if (!L[q].valid) break;
            cnt++;
            if (first_untouched < 0) {
                int is_t = 0;
                for (t = 0; t < *ntouched; t++) if (touched[t].idx == L[q].idx) { is_t = 1; break; }
                if (!is_t) first_untouched = q;
            }
        }
        out_feas[i] = (int32_t)fc;
        if (fc == 0) { out_idx[i] = OR_NO_FIT; out_score[i] = 0.0; continue; }
        if (first_untouched >= 0) {
            const or_rec *u = &L[first_untouched];
            if (tb >= 0 && cand_better(tkey, touched[tb].idx, u->key, u->idx)) { w = touched[tb].idx; wkey = tkey; }
            else { w = u->idx; wkey = u->key; }
        } else if (cnt < K) {
            if (tb >= 0) { w = touched[tb].idx; wkey = tkey; }
        } else {
            if (tb >= 0 && cand_better(tkey, touched[tb].idx, L[K - 1].key, L[K - 1].idx)) { w = touched[tb].idx; wkey = tkey; }
            else if (!rs || (rs->max_per_batch >= 0 && rs->in_batch >= rs->max_per_batch))
                return i; /* overflow: the best untouched node may lie beyond the list */
            else {
                /* rescue: the best node outside the touched set over every node, at its current state -- per
                 * shard (each rank scans its own rows), then the best of the shards' results */
                int64_t bj = -1;
                double bk = 0.0;
                int ul = o->use_labels && rs->labels && sel;
                int32_t r, R = rs->shards > 0 ? rs->shards : 1;
                for (r = 0; r < R; r++) {
                    double k = 0.0;
                    const int64_t lo = rs->n * r / R, hi = rs->n * (r + 1) / R;
                    const int64_t j = rescue_scan(o, rs, lo, hi, rc[i], rm[i], rp[i], s, ul, touched, *ntouched, &k);
                    if (j >= 0 && (bj < 0 || cand_better(k, j, bk, bj))) { bk = k; bj = j; }
                }
                rs->count++;
                rs->in_batch++;
                if (tb >= 0 && (bj < 0 || cand_better(tkey, touched[tb].idx, bk, bj))) { w = touched[tb].idx; wkey = tkey; }
                else if (bj >= 0) { w = bj; wkey = bk; rj = bj; }
            }
        }
        if (w < 0) { out_idx[i] = OR_NO_POSITIVE_SCORE; out_score[i] = 0.0; continue; }
        /* commit */
        {
            int32_t slot = -1;
            for (t = 0; t < *ntouched; t++) if (touched[t].idx == w) { slot = t; break; }
            if (slot < 0 && rj >= 0) { /* the rescued node: its state from the rows */
                if (*ntouched >= max_touched) return i;
                slot = (*ntouched)++;
                touched[slot].idx = (int32_t)rj;
                touched[slot].s0[0] = touched[slot].cur[0] = rs->ac[rj];
                touched[slot].s0[1] = touched[slot].cur[1] = rs->am[rj];
                touched[slot].s0[2] = touched[slot].cur[2] = rs->ap[rj];
                touched[slot].labels = rs->labels ? rs->labels[rj] : 0;
                touched[slot].price = rs->price ? rs->price[rj] : 0.f;
            }
            if (slot < 0) {
                const or_rec *u = NULL;
                for (q = 0; q < cnt; q++) if (L[q].idx == w) { u = &L[q]; break; }
                if (!u || *ntouched >= max_touched) return i; /* cannot happen: winner not touched comes from the list */
                slot = (*ntouched)++;
                touched[slot].idx = (int32_t)w;
                touched[slot].s0[0] = touched[slot].cur[0] = u->a_cpu;
                touched[slot].s0[1] = touched[slot].cur[1] = u->a_mem;
                touched[slot].s0[2] = touched[slot].cur[2] = u->a_pods;
                touched[slot].labels = u->labels;
                touched[slot].price = u->price;
            }
            touched[slot].cur[0] = wsub(touched[slot].cur[0], rc[i]);
            touched[slot].cur[1] = wsub(touched[slot].cur[1], rm[i]);
            touched[slot].cur[2] = wsub(touched[slot].cur[2], 1);
            out_idx[i] = (int32_t)w;
            out_score[i] = out_score_of(o, wkey);
        }
    }
    return nb;
}

/* Whole batched schedule on one shard (R = 1).  stats[0] = batches, stats[1] = truncations,
 * stats[2] = pairs evaluated in score passes. */
int or_schedule_batched(const or_opts *o, int32_t K, int32_t B, int64_t n,
                        int64_t *ac, int64_t *am, int64_t *ap, const uint64_t *labels, const float *price,
                        int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                        int32_t *out_idx, double *out_score, int32_t *out_feas, int64_t *stats)
{
    int64_t pos = 0;
    or_rec *recs;
    int64_t *fc;
    or_touched *touched;
    if (K < 1 || B < 1) return OR_E_INVALID;
    recs = (or_rec *)malloc(sizeof(or_rec) * (size_t)K * (size_t)B);
    fc = (int64_t *)malloc(sizeof(int64_t) * (size_t)B);
    touched = (or_touched *)malloc(sizeof(or_touched) * (size_t)B);
    if (!recs || !fc || !touched) { free(recs); free(fc); free(touched); return OR_E_INVALID; }
    if (stats) stats[0] = stats[1] = stats[2] = 0;
    while (pos < p) {
        int64_t nb = p - pos < B ? p - pos : B, done;
        int32_t nt = 0, t;
        or_local_topk(o, K, 0, n, ac, am, ap, labels, price, nb, rc + pos, rm + pos, rp + pos,
                      sel ? sel + pos : NULL, recs, fc);
        done = or_commit_batch(o, K, nb, rc + pos, rm + pos, rp + pos, sel ? sel + pos : NULL, recs, fc,
                               touched, &nt, B, out_idx + pos, out_score + pos, out_feas + pos);
        for (t = 0; t < nt; t++) {
            ac[touched[t].idx] = touched[t].cur[0];
            am[touched[t].idx] = touched[t].cur[1];
            ap[touched[t].idx] = touched[t].cur[2];
        }
        if (stats) { stats[0]++; stats[1] += done < nb; stats[2] += nb * n; }
        pos += done;
    }
    free(recs); free(fc); free(touched);
    return OR_OK;
}

int or_rec_size(void) { return (int)sizeof(or_rec); }
int or_touched_size(void) { return (int)sizeof(or_touched); }

/* ------------------------------------------------------------------------------------------ */
/* Pipelined restatement of the GPU batched mode: batch b is scored against */
/* the node rows as of batch b-2's commits (lag one batch), speculatively planned at the previous */
/* start + B; commit(b) skips a batch whose planned start is not the committed frontier, inherits */
/* the nodes committed by batch b-1, and stops at the first candidate-list overflow (resync).    */
/* ------------------------------------------------------------------------------------------ */

typedef struct or_xrec { int32_t idx; int64_t sb[3], cur[3]; uint64_t labels; float price; } or_xrec;

static int64_t commit_inherit(const or_opts *o, int32_t K, int64_t nb, const int64_t *rc, const int64_t *rm,
                              const int64_t *rp, const uint64_t *sel, const or_rec *lists, const int64_t *fc0,
                              const or_xrec *xin, int32_t nin, or_xrec *xout, int32_t *nout,
                              int32_t *out_idx, double *out_score, int32_t *out_feas, or_rescue *rs)
{
    /* touched table: inherited entries first (s0 = state at this batch's snapshot, cur = current) */
    or_touched *T = (or_touched *)malloc(sizeof(or_touched) * (size_t)(nin + nb + 1));
    int32_t *mine = (int32_t *)calloc((size_t)(nin + nb + 1), sizeof(int32_t));
    int64_t (*sb)[3] = malloc(sizeof(int64_t[3]) * (size_t)(nin + nb + 1));
    int32_t nt = nin, t;
    int64_t done;
    for (t = 0; t < nin; t++) {
        T[t].idx = xin[t].idx;
        memcpy(T[t].s0, xin[t].sb, sizeof(T[t].s0));
        memcpy(T[t].cur, xin[t].cur, sizeof(T[t].cur));
        memcpy(sb[t], xin[t].cur, sizeof(sb[t]));
        T[t].labels = xin[t].labels; T[t].price = xin[t].price;
    }
    {
        /* reuse or_commit_batch's decision rule, but with a pre-filled touched table */
        int32_t before = nt;
        done = commit_batch_impl(o, K, nb, rc, rm, rp, sel, lists, fc0, T, &nt, nin + (int32_t)nb + 1,
                                 out_idx, out_score, out_feas, rs);
        /* entries opened by this batch: state at batch start = snapshot state */
        for (t = before; t < nt; t++) memcpy(sb[t], T[t].s0, sizeof(sb[t]));
    }
    /* which entries did this batch commit to?  an entry changed iff cur != state at batch start */
    *nout = 0;
    for (t = 0; t < nt; t++) {
        int64_t i;
        int hit = t >= nin;
        for (i = 0; !hit && i < done; i++) hit = out_idx[i] == T[t].idx;
        if (!hit) continue;
        xout[*nout].idx = T[t].idx;
        memcpy(xout[*nout].sb, sb[t], sizeof(sb[t]));
        memcpy(xout[*nout].cur, T[t].cur, sizeof(T[t].cur));
        xout[*nout].labels = T[t].labels; xout[*nout].price = T[t].price;
        (*nout)++;
    }
    (void)mine;
    free(T); free(mine); free(sb);
    return done;
}

int or_schedule_pipelined(const or_opts *o, int32_t K, int32_t B, int64_t n,
                          int64_t *ac, int64_t *am, int64_t *ap, const uint64_t *labels, const float *price,
                          int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                          int32_t *out_idx, double *out_score, int32_t *out_feas, int64_t *stats)
{
    /* ac/am/ap are the node rows (what score reads); they receive batch b-2's commits before batch b */
    or_xrec *X[3];
    int32_t nx[3] = {0, 0, 0};
    or_rec *recs;
    int64_t *fc;
    int64_t cursor = 0, spec_next = 0, b;
    int resync = 0, k;
    if (K < 1 || B < 1) return OR_E_INVALID;
    for (k = 0; k < 3; k++) X[k] = (or_xrec *)malloc(sizeof(or_xrec) * (size_t)(2 * B + 1));
    recs = (or_rec *)malloc(sizeof(or_rec) * (size_t)K * (size_t)B);
    fc = (int64_t *)malloc(sizeof(int64_t) * (size_t)B);
    if (stats) stats[0] = stats[1] = stats[2] = 0;
    for (b = 0; cursor < p; b++) {
        int cb = (int)(b % 3), pb = (int)((b + 2) % 3); /* X(b), X(b-1) */
        int64_t s, nb, done, i;
        if (b >= 2) { /* apply(b-2) */
            int ab = (int)((b - 2) % 3);
            for (i = 0; i < nx[ab]; i++) {
                int32_t j = X[ab][i].idx;
                ac[j] = X[ab][i].cur[0]; am[j] = X[ab][i].cur[1]; ap[j] = X[ab][i].cur[2];
            }
            nx[ab] = 0;
        }
        /* plan(b): sees the commits of batches <= b-2 */
        if (resync) { s = cursor; resync = 0; } else s = spec_next;
        spec_next = s + B;
        /* commit(b-1) happens "concurrently" with score(b): model it after plan(b) */
        (void)pb;
        nb = s < p ? (p - s < B ? p - s : B) : 0;
        if (nb > 0) or_local_topk(o, K, 0, n, ac, am, ap, labels, price, nb, rc + s, rm + s, rp + s,
                                  sel ? sel + s : NULL, recs, fc);
        /* commit(b) */
        nx[cb] = 0;
        if (nb == 0) continue;
        if (s != cursor) { if (stats) stats[2]++; continue; } /* invalidated speculation */
        done = commit_inherit(o, K, nb, rc + s, rm + s, rp + s, sel ? sel + s : NULL, recs, fc,
                              X[(b + 2) % 3], b >= 1 ? nx[(b + 2) % 3] : 0, X[cb], &nx[cb],
                              out_idx + s, out_score + s, out_feas + s, NULL);
        cursor = s + done;
        if (done < nb) resync = 1;
        if (stats) { stats[0]++; stats[1] += done < nb; }
    }
    /* drain: the last two batches' commits */
    for (k = 0; k < 3; k++) {
        int64_t i;
        int ab = (int)((b - 2 + k + 3) % 3);
        if (b - 2 + k < 0 || b - 2 + k >= b) continue;
        for (i = 0; i < nx[ab]; i++) {
            int32_t j = X[ab][i].idx;
            ac[j] = X[ab][i].cur[0]; am[j] = X[ab][i].cur[1]; ap[j] = X[ab][i].cur[2];
        }
    }
    for (k = 0; k < 3; k++) free(X[k]);
    free(recs); free(fc);
    return OR_OK;
}

/* The persistent pipeline at lag L (2 <= L <= 4; the device runs L = 3, ksched_pipe.hip): batch b is
 * scored against the node state after commit(b - L); commit(b) inherits the nodes committed by batches
 * b - L + 1 .. b - 1, each with its state at b's snapshot (the start state of the oldest of those batches
 * that committed it) and its current state (after the newest); plan(b) for b < L is b * B, commit(b)
 * plans batch b + L (its cursor after a truncation, else plan(b + L - 1) + B), and a batch whose plan is
 * not the cursor is skipped.  Test infrastructure: tests/test_oracle.py checks it against or_schedule. */
int or_schedule_lagged_rescue(const or_opts *o, int32_t K, int32_t B, int32_t L, int32_t rescue, int64_t n,
                              int64_t *ac, int64_t *am, int64_t *ap, const uint64_t *labels, const float *price,
                              int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp,
                              const uint64_t *sel, int32_t *out_idx, double *out_score, int32_t *out_feas,
                              int64_t *stats);

int or_schedule_lagged_rescue2(const or_opts *o, int32_t K, int32_t B, int32_t L, int32_t rescue_max,
                               int32_t shards, int64_t n, int64_t *ac, int64_t *am, int64_t *ap,
                               const uint64_t *labels, const float *price, int64_t p, const int64_t *rc,
                               const int64_t *rm, const int64_t *rp, const uint64_t *sel, int32_t *out_idx,
                               double *out_score, int32_t *out_feas, int64_t *stats);

int or_schedule_lagged(const or_opts *o, int32_t K, int32_t B, int32_t L, int64_t n,
                       int64_t *ac, int64_t *am, int64_t *ap, const uint64_t *labels, const float *price,
                       int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp, const uint64_t *sel,
                       int32_t *out_idx, double *out_score, int32_t *out_feas, int64_t *stats)
{
    return or_schedule_lagged_rescue(o, K, B, L, 0, n, ac, am, ap, labels, price, p, rc, rm, rp, sel, out_idx,
                                     out_score, out_feas, stats);
}

/* rescue = 1: an exhausted list is rescued by a full scan of the untouched nodes (or_rescue) instead of
 * truncating the batch -- the device's persistent commit since round 4; stats[3] = rescues. */
int or_schedule_lagged_rescue(const or_opts *o, int32_t K, int32_t B, int32_t L, int32_t rescue, int64_t n,
                              int64_t *ac, int64_t *am, int64_t *ap, const uint64_t *labels, const float *price,
                              int64_t p, const int64_t *rc, const int64_t *rm, const int64_t *rp,
                              const uint64_t *sel, int32_t *out_idx, double *out_score, int32_t *out_feas,
                              int64_t *stats)
{
    return or_schedule_lagged_rescue2(o, K, B, L, rescue ? -1 : 0, 1, n, ac, am, ap, labels, price, p, rc, rm, rp,
                                      sel, out_idx, out_score, out_feas, stats);
}

/* The same with the device's rescue budget and node sharding: rescue_max rescues per batch (0: none, < 0: no
 * limit; the next exhausted list truncates the batch), the rescue's scan split over `shards` contiguous node
 * shards whose results are folded (ksched_pipe.hip serve_rescue per rank + ksched_commit.h's rank fold). */
int or_schedule_lagged_rescue2(const or_opts *o, int32_t K, int32_t B, int32_t L, int32_t rescue_max,
                               int32_t shards, int64_t n, int64_t *ac, int64_t *am, int64_t *ap,
                               const uint64_t *labels, const float *price, int64_t p, const int64_t *rc,
                               const int64_t *rm, const int64_t *rp, const uint64_t *sel, int32_t *out_idx,
                               double *out_score, int32_t *out_feas, int64_t *stats)
{
    enum { RING = 8 };
    or_rescue rs = {n, ac, am, ap, labels, price, 0, shards < 1 ? 1 : shards, rescue_max, 0};
    const int rescue = rescue_max != 0;
    or_xrec *X[RING], *inh;
    int32_t nx[RING];
    int64_t plan[RING];
    or_rec *recs;
    int64_t *fc;
    int64_t cursor = 0, b;
    int k;
    if (K < 1 || B < 1 || L < 2 || L > 4) return OR_E_INVALID;
    for (k = 0; k < RING; k++) { X[k] = (or_xrec *)malloc(sizeof(or_xrec) * (size_t)(B + 1)); nx[k] = 0; plan[k] = -1; }
    inh = (or_xrec *)malloc(sizeof(or_xrec) * (size_t)(L * B + 1));
    recs = (or_rec *)malloc(sizeof(or_rec) * (size_t)K * (size_t)B);
    fc = (int64_t *)malloc(sizeof(int64_t) * (size_t)B);
    for (k = 0; k < L; k++) plan[k] = (int64_t)k * B < p ? (int64_t)k * B : -1;
    if (stats) stats[0] = stats[1] = stats[2] = 0;
    for (b = 0; cursor < p; b++) {
        const int cb = (int)(b % RING);
        int64_t s = plan[cb], nb, done, i, nxt;
        int32_t nin = 0, t;
        int d;
        if (b >= L) { /* score(b) sees commit(b - L) */
            const int ab = (int)((b - L) % RING);
            for (i = 0; i < nx[ab]; i++) {
                const int32_t j = X[ab][i].idx;
                ac[j] = X[ab][i].cur[0]; am[j] = X[ab][i].cur[1]; ap[j] = X[ab][i].cur[2];
            }
        }
        nx[cb] = 0;
        nb = (s >= 0 && s < p) ? (p - s < B ? p - s : B) : 0;
        if (nb > 0) or_local_topk(o, K, 0, n, ac, am, ap, labels, price, nb, rc + s, rm + s, rp + s,
                                  sel ? sel + s : NULL, recs, fc);
        if (nb == 0 || s != cursor) {
            if (nb > 0 && stats) stats[2]++; /* invalidated speculation */
            nxt = plan[(b + L - 1) % RING];
            plan[(b + L) % RING] = nxt < 0 || nxt + B >= p ? -1 : nxt + B;
            continue;
        }
        /* inherited: newest export first; an older export's entry for a node already present only
         * moves that node's snapshot state back to the older start state */
        for (d = 1; d < L && b - d >= 0; d++) {
            const int xb = (int)((b - d) % RING);
            for (i = 0; i < nx[xb]; i++) {
                for (t = 0; t < nin && inh[t].idx != X[xb][i].idx; t++) {}
                if (t == nin) inh[nin++] = X[xb][i];
                else memcpy(inh[t].sb, X[xb][i].sb, sizeof(inh[t].sb));
            }
        }
        done = commit_inherit(o, K, nb, rc + s, rm + s, rp + s, sel ? sel + s : NULL, recs, fc, inh, nin,
                              X[cb], &nx[cb], out_idx + s, out_score + s, out_feas + s, rescue ? &rs : NULL);
        cursor = s + done;
        nxt = plan[(b + L - 1) % RING];
        nxt = done < nb ? cursor : (nxt < 0 ? -1 : nxt + B);
        plan[(b + L) % RING] = nxt >= p ? -1 : nxt;
        if (stats) { stats[0]++; stats[1] += done < nb; }
    }
    /* drain: the commits the last batches' scores never saw */
    for (k = L; k >= 1; k--) {
        int64_t i;
        const int ab = (int)((b - k) % RING);
        if (b - k < 0) continue;
        for (i = 0; i < nx[ab]; i++) {
            const int32_t j = X[ab][i].idx;
            ac[j] = X[ab][i].cur[0]; am[j] = X[ab][i].cur[1]; ap[j] = X[ab][i].cur[2];
        }
    }
    if (stats) stats[3] = rs.count;
    for (k = 0; k < RING; k++) free(X[k]);
    free(inh); free(recs); free(fc);
    return OR_OK;
}
