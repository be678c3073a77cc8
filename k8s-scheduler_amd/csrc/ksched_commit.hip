// ksched_commit.hip -- ordered commit of one speculative batch, lane = pod (gfx950).
//
// The sequential semantics (anchor/schedule.go:185-197: every pod sees the placements of the pods
// before it) are replayed by one wave in pod order, but the per-pod work is spread across the lanes
// by POD rather than by touched node: lane j owns pod j of the batch and keeps, in LDS, its score
// against every touched node (S[j][t], t = touched slot).  A commit changes exactly one node, so
// after pod i commits to node w the whole wave re-scores w for all pods at once (one exact score per
// lane) and updates every pod's predicate count and first-untouched candidate.  Pod i+1's decision is
// then one LDS row read + a wave arg-best, instead of re-scoring the whole touched set per pod.
//
// Definitions (same as the single-wave sequencer k_commit):
//   T    = nodes whose state may differ from the batch's score snapshot: the previous batch's
//          commits (inherited from its XBuf) plus this batch's commits so far;
//   fc_j = fc0_j - sum_T fits(j, s0) + sum_T fits(j, cur)        (predicate.go:127-150 count)
//   u*_j = first entry of pod j's list not in T (its key is exact: untouched since the snapshot)
//   t*_j = best of T at the current state (re-scored exactly)
//   winner = better(u*, t*); list exhausted and full: t* must beat list[K-1], else the batch stops
//   before pod i (truncation; the pipeline resyncs at the cursor).
#include <hip/hip_runtime.h>

#include "ksched_kernels.h"

namespace ksched {

namespace {

constexpr int kLpRow = kLpSlots + 1;  // S row stride (doubles): row writes and column reads conflict-free

struct LpSmem {
    int32_t *hkey;    // open-addressed set of touched node indices (-1 = empty)
    uint32_t *filt;   // 64K-bit filter in front of the hash
    int32_t *ti;      // node index per touched slot
    int32_t *dfacc;   // per pod: sum over inherited slots of fits(cur) - fits(s0)
    uint32_t *tm;     // per pod: bit q = list entry q's node is inherited (in T at the start)
    Touched *T;       // touched slots
    double *S;        // [64 pods][kLpRow] key of (pod, slot); -inf = not eligible
    CandStage *CS;    // [64 pods][K] staged candidate lists (node snapshot state; wave-uniform reads)
    double *LK;       // [K][64] candidate keys, lane-contiguous (per-lane pointer walks are conflict-free)
    int32_t *LI;      // [K][64] candidate node indices
};

__device__ __forceinline__ uint32_t lp_hash(int32_t idx) { return ((uint32_t)idx * 2654435761u) >> (32 - kTouchHashBits); }

__device__ __forceinline__ bool lp_has(const LpSmem &m, int32_t idx) {
    if (!(m.filt[((uint32_t)idx & 0xffffu) >> 5] & (1u << ((uint32_t)idx & 31)))) return false;
    for (uint32_t h = lp_hash(idx);; h = (h + 1) & (kTouchHash - 1)) {
        const int32_t k = m.hkey[h];
        if (k == idx) return true;
        if (k < 0) return false;
    }
}

__device__ __forceinline__ double uniform_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, int src) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)v >> 32), src);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// diagnostics (KSCHED_COMMIT_STAMPS): shader-clock stamp, ordered against the surrounding code
__device__ __forceinline__ uint64_t lp_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

}  // namespace

template <int K, int PRIO, int DOM, bool LAB, bool F53, bool ST>
__global__ __launch_bounds__(kLpThreads) void k_commit_lp(CommitArgs A) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical: win issue arbitration over co-resident score waves
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    constexpr int nw = kLpThreads / 64;
    const int64_t p0 = *A.plan;
    const int64_t cursor = A.ctl->cursor;
    if (p0 < 0 || p0 >= A.pods.p || p0 != cursor) {
        // nothing to do, or a speculative batch invalidated by an earlier truncation: skip it
        if (tid == 0) {
            A.xout->count = 0;
            if (p0 >= 0 && p0 < A.pods.p) A.ctl->stats[3] += 1;
            plan_after_commit(A, false, cursor);
        }
        return;
    }
    uint64_t tp0 = 0, ph[6] = {0, 0, 0, 0, 0, 0};
    if (ST) tp0 = lp_stamp();
    LpSmem m;
    char *p = smem;
    m.hkey = reinterpret_cast<int32_t *>(p); p += kTouchHash * sizeof(int32_t);
    m.filt = reinterpret_cast<uint32_t *>(p); p += kTouchFilterWords * sizeof(uint32_t);
    m.ti = reinterpret_cast<int32_t *>(p); p += kLpSlots * sizeof(int32_t);
    m.dfacc = reinterpret_cast<int32_t *>(p); p += 64 * sizeof(int32_t);
    m.tm = reinterpret_cast<uint32_t *>(p); p += 64 * sizeof(uint32_t);
    m.T = reinterpret_cast<Touched *>(p); p += kLpSlots * sizeof(Touched);
    m.S = reinterpret_cast<double *>(p); p += (size_t)64 * kLpRow * sizeof(double);
    m.CS = reinterpret_cast<CandStage *>(p); p += (size_t)64 * K * sizeof(CandStage);
    m.LK = reinterpret_cast<double *>(p); p += (size_t)64 * K * sizeof(double);
    m.LI = reinterpret_cast<int32_t *>(p);
    const int nb = (int)((A.pods.p - p0 < A.B) ? A.pods.p - p0 : A.B);  // <= 64 (host-checked)

    // ---- prologue (all waves): stage lists, inherit the previous batch's commits ----
    for (int w = tid; w < kTouchHash; w += kLpThreads) m.hkey[w] = -1;
    for (int w = tid; w < kTouchFilterWords; w += kLpThreads) m.filt[w] = 0;
    if (tid < 64) { m.dfacc[tid] = 0; m.tm[tid] = 0; }
    for (int e = tid; e < nb * K; e += kLpThreads) {
        const Rec r = A.lists[e];
        CandStage c;
        c.key = r.key; c.idx = r.valid ? r.idx : kNoIdx; c.price = r.price;
        c.a[0] = r.a[0]; c.a[1] = r.a[1]; c.a[2] = r.a[2]; c.labels = r.labels;
        m.CS[e] = c;
        m.LK[(e % K) * 64 + e / K] = c.key;
        m.LI[(e % K) * 64 + e / K] = c.idx;
    }
    __syncthreads();
    const int nin = A.xin->count;
    for (int e = tid; e < nin; e += kLpThreads) {
        const XRec &xi = A.xin->e[e];
        Touched &x = m.T[e];
        x.idx = xi.idx; x.mine = 0;
        for (int r = 0; r < 3; ++r) {
            x.s0[r] = xi.sb[r];   // state at this batch's score snapshot
            x.sb[r] = xi.cur[r];  // state when this batch's commit starts
            x.cur[r] = xi.cur[r];
            x.curf[r] = (double)xi.cur[r];
            x.cury[r] = recip_or_zero(xi.cur[r], x.curf[r]);
        }
        x.labels = xi.labels; x.price = xi.price; x.pad2 = 0;
        m.ti[e] = xi.idx;
        uint32_t h = lp_hash(xi.idx);
        while (atomicCAS(&m.hkey[h], -1, xi.idx) != -1) h = (h + 1) & (kTouchHash - 1);
        atomicOr(&m.filt[((uint32_t)xi.idx & 0xffffu) >> 5], 1u << ((uint32_t)xi.idx & 31));
    }
    __syncthreads();

    // lane = pod j of the batch (lanes >= nb carry a zero request and are never read)
    const bool pj = lane < nb;
    const int64_t rc = pj ? A.pods.rc[p0 + lane] : 0;
    const int64_t rm = pj ? A.pods.rm[p0 + lane] : 0;
    const int64_t rp = pj ? A.pods.rp[p0 + lane] : 0;
    const uint64_t sel = (LAB && pj) ? A.pods.sel[p0 + lane] : 0;
    const double rcf = (double)rc, rmf = (double)rm, rpf = (double)rp;
    const double y3 = recip(3.0);
    double *Srow = m.S + (size_t)lane * kLpRow;

    // inherited slots (all waves): every pod's key against the slot's current state, its predicate
    // delta and a per-wave partial row best; list entry q's touched bit by wave q.  Columns 64..95 of
    // S are free during the prologue (inherited slots < 64) and hold the partial row bests.
    {
        int dfl = 0;
        double pk = -__builtin_inf();
        int32_t pi = kNoIdx, ps = -1;
        for (int t = wave; t < nin; t += nw) {
            const Touched &x = m.T[t];
            const bool f0 = fits(rc, rm, rp, sel, x.s0[0], x.s0[1], x.s0[2], x.labels, LAB);
            const bool f1 = fits(rc, rm, rp, sel, x.cur[0], x.cur[1], x.cur[2], x.labels, LAB);
            dfl += (int)f1 - (int)f0;
            double k;
            const bool el = pair_key_fast<PRIO, DOM, F53>(f1, rc, rm, rp, rcf, rmf, rpf, x.cur[0], x.cur[1], x.cur[2],
                                                          x.curf[0], x.curf[1], x.curf[2], x.cury[0], x.cury[1],
                                                          x.cury[2], y3, x.price, &k);
            k = el ? k : -__builtin_inf();
            Srow[t] = k;
            const bool up = el && better(k, m.ti[t], pk, pi);
            pk = up ? k : pk;
            pi = up ? m.ti[t] : pi;
            ps = up ? t : ps;
        }
        if (wave < nin) {
            Srow[64 + wave] = pk;
            reinterpret_cast<int64_t *>(Srow)[80 + wave] = ((int64_t)ps << 32) | (uint32_t)pi;
        }
        if (dfl != 0) atomicAdd(&m.dfacc[lane], dfl);
        if (nin > 0 && wave < K && pj) {
            const int32_t x = m.LI[wave * 64 + lane];
            if (x != kNoIdx && lp_has(m, x)) atomicOr(&m.tm[lane], 1u << wave);
        }
    }
    __syncthreads();
    if (wave != 0) return;

    // ---- sequencer (wave 0 alone; no barriers from here on) ----
    // Per lane j (pod j): fc (predicate count), the list (node indices in registers, keys in LDS),
    // tmask (bit q: list entry q's node is in T), ptr (first untouched entry = u*), and the running
    // best of row j of S (rbk, rbi, rbs).  A commit only ever changes one column of S, so the running
    // best stays exact unless the column holding it got worse ("dirty"); only then is row i
    // re-reduced across the wave when pod i's turn comes.
    int32_t fc = pj ? (int32_t)(A.fc0[lane] + m.dfacc[lane]) : 0;  // <= nodes < 2^31
    const int cut = pj ? A.lists[(size_t)lane * K].pad : 0;  // unlisted candidates rank below the last entry
    const double *LKl = m.LK + lane;  // entry q of this lane's list at [q * 64]
    const int32_t *LIl = m.LI + lane;
    int32_t li[K];
    int cv = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) {
        li[q] = pj ? LIl[q * 64] : kNoIdx;
        cv += li[q] != kNoIdx;  // valid entries form a prefix
    }
    const uint32_t vmask = (1u << cv) - 1u;  // cv <= 16
    uint32_t tmask = m.tm[lane];
    int ptr = __builtin_ctz((~tmask & vmask) | (1u << cv));
    double uk = ptr < cv ? LKl[ptr * 64] : -__builtin_inf();
    int32_t ui = ptr < cv ? LIl[ptr * 64] : kNoIdx;
    double rbk = -__builtin_inf();
    int32_t rbi = kNoIdx, rbs = -1;
    bool dirty = false;
    {
        const int nwp = nin < nw ? nin : nw;
        for (int w = 0; w < nwp; ++w) {
            const double k = Srow[64 + w];
            const int64_t pk = reinterpret_cast<const int64_t *>(Srow)[80 + w];
            const int32_t x = (int32_t)(uint32_t)pk;
            if (k != -__builtin_inf() && better(k, x, rbk, rbi)) { rbk = k; rbi = x; rbs = (int32_t)(pk >> 32); }
        }
    }
    // this lane's pod outcome, captured at its turn and stored once at the end
    int32_t my_idx = 0, my_feas = 0;
    double my_score = 0.0;

    int nT = nin;
    int64_t placed = 0, nred = 0, nk1 = 0;
    int done = nb;
    uint64_t ta = 0, tb = 0;
    if (ST) { ta = lp_stamp(); ph[0] = ta - tp0; }
    for (int i = 0; i < nb; ++i) {
        // t*: best touched node for pod i at the current state
        double tk;
        int32_t ti, ts;
        if (__builtin_amdgcn_readlane((int)dirty, i) == 0) {
            tk = readlane_f64(rbk, i);
            ti = __builtin_amdgcn_readlane(rbi, i);
            ts = __builtin_amdgcn_readlane(rbs, i);
        } else {
            ++nred;
            const double *Si = m.S + (size_t)i * kLpRow;
            const double k0 = Si[lane], k1 = Si[lane + 64];
            const int32_t x0 = m.ti[lane], x1 = m.ti[lane + 64];
            const bool e0 = lane < nT && k0 != -__builtin_inf();
            const bool e1 = lane + 64 < nT && k1 != -__builtin_inf();
            tk = e0 ? k0 : -__builtin_inf();
            ti = e0 ? x0 : kNoIdx;
            ts = e0 ? lane : -1;
            const bool b1 = e1 && better(k1, x1, tk, ti);
            tk = b1 ? k1 : tk;
            ti = b1 ? x1 : ti;
            ts = b1 ? lane + 64 : ts;
            wave_argbest_fast(tk, ti, ts);
        }
        tk = uniform_f64(tk);
        ti = __builtin_amdgcn_readfirstlane(ti);
        ts = __builtin_amdgcn_readfirstlane(ts);
        if (ST) { tb = lp_stamp(); ph[1] += tb - ta; ta = tb; }
        const int32_t fci = __builtin_amdgcn_readlane(fc, i);
        const int pi = __builtin_amdgcn_readlane(ptr, i);
        const int cvi = __builtin_amdgcn_readlane(cv, i);
        const int cuti = __builtin_amdgcn_readlane(cut, i);
        const double uki = readlane_f64(uk, i);
        const int32_t uii = __builtin_amdgcn_readlane(ui, i);
        int kind = 0;  // 0 no candidate, 1 list entry (first touch), 2 touched node, 3 overflow
        const bool has_t = ti != kNoIdx;
        if (fci != 0) {
            if (pi < cvi) {
                kind = (has_t && better(tk, ti, uki, uii)) ? 2 : 1;
            } else if (!cuti) {
                kind = has_t ? 2 : 0;
            } else if (cvi > 0) {
                // every unlisted untouched node ranks below the last valid entry
                const double lk = m.LK[(cvi - 1) * 64 + i];
                const int32_t lx = m.LI[(cvi - 1) * 64 + i];
                kind = (has_t && better(tk, ti, lk, lx)) ? 2 : 3;
            } else {
                kind = 3;  // unreachable: a cut list keeps at least its cutoff entry
            }
        }
        kind = __builtin_amdgcn_readfirstlane(kind);
        if (ST) { tb = lp_stamp(); ph[2] += tb - ta; ta = tb; }
        if (kind == 3) { done = i; break; }  // overflow: stop before pod i (wave-uniform)
        int32_t oidx = fci == 0 ? -1 : -2;   // NO_FIT (schedule.go:74-76) / NO_POSITIVE_SCORE (priorities.go:55-62)
        double osc = 0.0;
        if (kind != 0) {
            const double wk = kind == 1 ? uki : tk;
            const int32_t wi = kind == 1 ? uii : ti;
            oidx = wi;
            osc = PRIO == kPrioPrice ? 0.0 - wk : wk;
            ++placed;
            int s;
            int64_t b0, b1, b2;
            uint64_t lab;
            float pr;
            if (kind == 1) {
                ++nk1;
                const CandStage &c = m.CS[(size_t)i * K + pi];
                b0 = c.a[0]; b1 = c.a[1]; b2 = c.a[2]; lab = c.labels; pr = c.price;
                s = nT++;
            } else {
                s = ts;
                const Touched &x = m.T[s];
                b0 = x.cur[0]; b1 = x.cur[1]; b2 = x.cur[2]; lab = x.labels; pr = x.price;
            }
            // commit: used += request, ONE pod (anchor/predicate.go:99-102)
            const int64_t n0 = wsub(b0, readlane_i64(rc, i)), n1 = wsub(b1, readlane_i64(rm, i)), n2 = wsub(b2, 1);
            const double nf0 = (double)n0, nf1 = (double)n1, nf2 = (double)n2;
            const double ny0 = recip_or_zero(n0, nf0), ny1 = recip_or_zero(n1, nf1), ny2 = recip_or_zero(n2, nf2);
            // every pod's view of node wi: predicate delta and exact key at the new state
            const bool fo = fits(rc, rm, rp, sel, b0, b1, b2, lab, LAB);
            const bool fn = fits(rc, rm, rp, sel, n0, n1, n2, lab, LAB);
            fc += (int32_t)fn - (int32_t)fo;
            double k;
            const bool el = pair_key_fast<PRIO, DOM, F53>(fn, rc, rm, rp, rcf, rmf, rpf, n0, n1, n2, nf0, nf1, nf2, ny0,
                                                          ny1, ny2, y3, pr, &k);
            Srow[s] = el ? k : -__builtin_inf();
            // running row best: a better value takes over; the holder getting worse marks the row dirty
            const bool up = el && better(k, wi, rbk, rbi);
            dirty = dirty || (!up && rbs == s);
            rbk = up ? k : rbk;
            rbi = up ? wi : rbi;
            rbs = up ? s : rbs;
            if (lane == 0) {
                Touched &x = m.T[s];
                if (kind == 1) {
                    x.idx = wi;
                    x.sb[0] = b0; x.sb[1] = b1; x.sb[2] = b2;  // untouched by the previous batch
                    x.labels = lab; x.price = pr; x.pad2 = 0;
                    m.ti[s] = wi;
                }
                x.mine = 1;
                x.cur[0] = n0; x.cur[1] = n1; x.cur[2] = n2;
            }
            if (ST) { tb = lp_stamp(); ph[3] += tb - ta; ta = tb; }
            if (kind == 1) {
                // node wi joins T: every list holding it marks the entry; u* moves to the next free one
#pragma unroll
                for (int q = 0; q < K; ++q) tmask |= (li[q] == wi) ? (1u << q) : 0u;
                const int np = __builtin_ctz((~tmask & vmask) | (1u << cv));
                if (np != ptr) {
                    ptr = np;
                    uk = ptr < cv ? LKl[ptr * 64] : -__builtin_inf();
                    ui = ptr < cv ? LIl[ptr * 64] : kNoIdx;
                }
            }
        }
        if (lane == i) { my_idx = oidx; my_score = osc; my_feas = fci; }
        if (ST) { tb = lp_stamp(); ph[4] += tb - ta; ta = tb; }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < done) {
        A.out.idx[p0 + lane] = my_idx;
        A.out.score[p0 + lane] = my_score;
        A.out.feas[p0 + lane] = my_feas;
    }
    // export this batch's commits (wave-ordered compaction)
    int base = 0;
    for (int t0 = 0; t0 < nT; t0 += 64) {
        const int t = t0 + lane;
        const bool mine = t < nT && m.T[t].mine;
        const uint64_t mask = __ballot(mine);
        if (mine) {
            const Touched &x = m.T[t];
            XRec &o = A.xout->e[base + __popcll(mask & ((1ull << lane) - 1))];
            o.idx = x.idx; o.pad = 0;
            o.sb[0] = x.sb[0]; o.sb[1] = x.sb[1]; o.sb[2] = x.sb[2];
            o.cur[0] = x.cur[0]; o.cur[1] = x.cur[1]; o.cur[2] = x.cur[2];
            o.labels = x.labels; o.price = x.price; o.pad2 = 0;
        }
        base += __popcll(mask);
    }
    if (lane == 0) {
        A.xout->count = base;
        A.ctl->cursor = p0 + done;
        A.ctl->stats[0] += 1;
        A.ctl->stats[1] += (done < nb) ? 1 : 0;
        A.ctl->stats[2] += placed;
        plan_after_commit(A, done < nb, p0 + done);
        if (ST) {
            A.dbg[0] += ph[0]; A.dbg[1] += ph[1]; A.dbg[2] += ph[2]; A.dbg[3] += ph[3]; A.dbg[4] += ph[4];
            A.dbg[5] += done; A.dbg[6] += nT; A.dbg[7] += 1; A.dbg[8] += lp_stamp() - tp0;
            A.dbg[9] += nred; A.dbg[10] += nk1; A.dbg[11] += placed;
        }
    }
}

namespace {

template <int K, int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_lp_one(const CommitArgs &a, hipStream_t s) {
    static bool attr_set = false;
    const size_t lds = commit_lp_lds_bytes(K);
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void *)k_commit_lp<K, PRIO, DOM, LAB, F53, false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void *)k_commit_lp<K, PRIO, DOM, LAB, F53, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (a.dbg) hipLaunchKernelGGL((k_commit_lp<K, PRIO, DOM, LAB, F53, true>), dim3(1), dim3(kLpThreads), lds, s, a);
    else hipLaunchKernelGGL((k_commit_lp<K, PRIO, DOM, LAB, F53, false>), dim3(1), dim3(kLpThreads), lds, s, a);
    return hipGetLastError();
}

template <int PRIO, int DOM, bool LAB, bool F53>
hipError_t commit_lp_k(int K, const CommitArgs &a, hipStream_t s) {
    switch (K) {
        case 4: return commit_lp_one<4, PRIO, DOM, LAB, F53>(a, s);
        case 8: return commit_lp_one<8, PRIO, DOM, LAB, F53>(a, s);
        case 16: return commit_lp_one<16, PRIO, DOM, LAB, F53>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_commit_lp(int K, int prio, int dom, bool lab, bool f53, const CommitArgs &a, hipStream_t s) {
    if (a.B > 64) return hipErrorInvalidValue;
    KSCHED_DISPATCH(prio, dom, lab, f53, (commit_lp_k<P_, D_, L_, F_>(K, a, s)));
}

}  // namespace ksched
