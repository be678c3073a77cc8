/*
 * ksched_driver.c -- the Go shim's call sequence (integration/anchor_ksched.go), as a C program linked
 * against libksched.so, so that the sequence a maintainer would ship is compiled and run here (this
 * image has no Go toolchain).  It replaces the reference's schedulePods loop
 * (anchor/schedule.go:185-197) for one reconcile pass:
 *
 *   ksched_create -> ksched_load_nodes                      (getNodes/getPods + usedResource, once)
 *   loop:  ksched_schedule(pending[start:])                 (predicate + priorities for every pod, in order)
 *          ksched_explain_pod per NO_FIT pod, in the bind loop (FailedScheduling lines of the pod,
 *                                                            anchor/predicate.go:152-173)
 *          bind each placed pod in order                    (anchor/schedule.go:200-261)
 *          on a failed bind of pod i: the reference leaves pod i unbound and every later pod re-reads
 *          a cluster WITHOUT it, so the engine's commits of pods i.. (none bound yet) are undone with
 *          ksched_apply_delta and the pods after i are scheduled again: start = i + 1
 *   then bound-pod watch events (the apply_delta feed INTEGRATION.md describes): ADDED of a pod bound by another scheduler
 *          charges its node, DELETED of a bound pod frees it (ksched_apply_delta); ADDED of a pod this run
 *          bound is skipped (already committed); a pod bound to a node missing from the node list ends
 *          the program with KSCHED_E_UNKNOWN_NODE, as the reference's usedResource panics there
 *          (anchor/predicate.go:94-99)
 *
 * Watch mode (argv[6] = "watch"): the shim's schedulePodGPU for monitorUnscheduledPods (anchor/schedule.go:47-89):
 * the pending pods arrive one at a time, each is ONE ksched_schedule call of one pod, then explain_pod on NO_FIT
 * or its bind; a failed bind undoes that pod's commit (ksched_apply_delta) and the next pod goes on from there --
 * the same sequential semantics as the batch loop.  (The Go shim reloads the cluster per pod, as predicate()
 * recounts per call; here the engine keeps the state the reloads would give.)
 *
 * Input (argv[1]) and output (argv[2]) are flat little-endian files written / read by
 * tests/test_gpu_integration.py; argv[3..]: mode, topk, batch, "batch" | "watch".  The "API server" is simulated: a bind
 * of a pod listed in the input's fail set returns an error, every other bind succeeds.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ksched.h"

#define BIND_FAILED (-3)

static int read_all(FILE *f, void *p, size_t bytes) { return fread(p, 1, bytes, f) == bytes ? 0 : -1; }

static void die(ksched_ctx *c, const char *what, int rc) {
    fprintf(stderr, "ksched_driver: %s failed (%d): %s\n", what, rc, c ? ksched_last_error(c) : "");
    exit(2);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ksched_driver in.bin out.bin [mode topk batch]\n");
        return 1;
    }
    FILE *in = fopen(argv[1], "rb");
    if (!in) { perror("input"); return 1; }
    int64_t hdr[8]; /* n, p, nfail, priority, domain, use_labels, has_price, nevents */
    if (read_all(in, hdr, sizeof(hdr))) { fprintf(stderr, "bad header\n"); return 1; }
    const int64_t n = hdr[0], p = hdr[1], nfail = hdr[2], nev = hdr[7];
    int64_t *ac = malloc(8 * n), *am = malloc(8 * n), *ap = malloc(8 * n);
    uint64_t *lab = malloc(8 * n);
    float *price = malloc(4 * n);
    int64_t *rc = malloc(8 * p), *rm = malloc(8 * p), *rp = malloc(8 * p);
    uint64_t *sel = malloc(8 * p);
    int64_t *failset = malloc(8 * (nfail + 1));
    int64_t *ev = malloc(8 * 5 * (nev + 1)); /* {type 1 ADDED | 2 DELETED, node (-1: not in the node list), cpu, mem, ours} */
    if (read_all(in, ac, 8 * n) || read_all(in, am, 8 * n) || read_all(in, ap, 8 * n) || read_all(in, lab, 8 * n) ||
        read_all(in, price, 4 * n) || read_all(in, rc, 8 * p) || read_all(in, rm, 8 * p) || read_all(in, rp, 8 * p) ||
        read_all(in, sel, 8 * p) || read_all(in, failset, 8 * nfail) || read_all(in, ev, 8 * 5 * nev)) {
        fprintf(stderr, "short input\n");
        return 1;
    }
    fclose(in);
    char *bind_fails = calloc((size_t)p, 1);
    for (int64_t k = 0; k < nfail; ++k)
        if (failset[k] >= 0 && failset[k] < p) bind_fails[failset[k]] = 1;

    ksched_opts o;
    ksched_default_opts(&o);
    o.priority = (int32_t)hdr[3];
    o.domain = (int32_t)hdr[4];
    o.use_labels = (int32_t)hdr[5];
    o.mode = argc > 3 ? atoi(argv[3]) : KSCHED_MODE_BATCHED;
    o.topk = argc > 4 ? atoi(argv[4]) : 16;
    o.batch = argc > 5 ? atoi(argv[5]) : 64;
    ksched_ctx *ctx = NULL;
    int rcode;
    if ((rcode = ksched_create(&o, &ctx)) != KSCHED_OK) die(NULL, "ksched_create", rcode);
    if ((rcode = ksched_load_nodes(ctx, n, ac, am, ap, hdr[5] ? lab : NULL, hdr[6] ? price : NULL)) != KSCHED_OK)
        die(ctx, "ksched_load_nodes", rcode);

    int32_t *idx = malloc(4 * p), *feas = malloc(4 * p);
    double *score = malloc(8 * p);
    int64_t *counts = calloc((size_t)p * KSCHED_NUM_REASONS, 8);
    uint8_t *reason = malloc((size_t)(n > 0 ? n : 1));
    int64_t calls = 0, binds = 0, failed_binds = 0, undone = 0;
    const int watch = argc > 6 && strcmp(argv[6], "watch") == 0;
    for (int64_t i = 0; watch && i < p; ++i) {
        /* schedulePodGPU(pending pod i) */
        rcode = ksched_schedule(ctx, 1, rc + i, rm + i, rp + i, hdr[5] ? sel + i : NULL, idx + i, score + i, feas + i);
        if (rcode != KSCHED_OK) die(ctx, "ksched_schedule", rcode);
        ++calls;
        if (idx[i] == KSCHED_NO_FIT) {
            if ((rcode = ksched_explain_pod(ctx, 0, counts + i * KSCHED_NUM_REASONS, n > 0 ? reason : NULL)) != KSCHED_OK)
                die(ctx, "ksched_explain_pod", rcode);
            continue;
        }
        if (idx[i] < 0) continue;
        if (!bind_fails[i]) { ++binds; continue; }
        ++failed_binds;
        const int64_t one = 1;
        if ((rcode = ksched_apply_delta(ctx, 1, idx + i, rc + i, rm + i, &one)) != KSCHED_OK) die(ctx, "ksched_apply_delta", rcode);
        ++undone;
        idx[i] = BIND_FAILED;
    }
    int64_t start = watch ? p : 0;
    while (start < p) {
        const int64_t m = p - start;
        rcode = ksched_schedule(ctx, m, rc + start, rm + start, rp + start, hdr[5] ? sel + start : NULL, idx + start,
                                score + start, feas + start);
        if (rcode != KSCHED_OK) die(ctx, "ksched_schedule", rcode);
        ++calls;
        int64_t resume = -1;
        for (int64_t i = start; i < p; ++i) {
            if (idx[i] == KSCHED_NO_FIT) {  /* FailedScheduling event for this pod (its turn's state) */
                /* the shim's failedSchedulingEvent: per-node reasons of pod i - start of this call */
                if ((rcode = ksched_explain_pod(ctx, i - start, counts + i * KSCHED_NUM_REASONS, n > 0 ? reason : NULL)) !=
                    KSCHED_OK)
                    die(ctx, "ksched_explain_pod", rcode);
                continue;
            }
            if (idx[i] < 0) continue; /* KSCHED_NO_POSITIVE_SCORE: the reference would panic in bind */
            if (!bind_fails[i]) { ++binds; continue; }
            /* bind(pod i) failed: undo the commits of pod i and of every later placement of this call */
            ++failed_binds;
            int64_t k = 0;
            for (int64_t j = i; j < p; ++j) k += idx[j] >= 0;
            int32_t *ui = malloc(4 * k);
            int64_t *dc = malloc(8 * k), *dm = malloc(8 * k), *dp = malloc(8 * k);
            k = 0;
            for (int64_t j = i; j < p; ++j) {
                if (idx[j] < 0) continue;
                ui[k] = idx[j]; dc[k] = rc[j]; dm[k] = rm[j]; dp[k] = 1; ++k;
            }
            if ((rcode = ksched_apply_delta(ctx, k, ui, dc, dm, dp)) != KSCHED_OK) die(ctx, "ksched_apply_delta", rcode);
            undone += k;
            free(ui); free(dc); free(dm); free(dp);
            idx[i] = BIND_FAILED;
            resume = i + 1;
            break;
        }
        if (resume < 0) break;
        start = resume;
    }
    /* bound-pod watch events fed to ksched_apply_delta ("Pods bound or deleted by others") */
    for (int64_t e = 0; e < nev; ++e) {
        const int64_t *x = ev + 5 * e;
        if (x[0] == 1 && x[4]) continue; /* ADDED for a pod this run bound: committed by ksched_schedule */
        if (x[1] < 0) {
            fprintf(stderr, "ksched_driver: watch event %lld: pod bound to an unknown node (%d)\n", (long long)e,
                    KSCHED_E_UNKNOWN_NODE);
            exit(-KSCHED_E_UNKNOWN_NODE);
        }
        const int64_t sign = x[0] == 2 ? 1 : -1; /* bound: used += (cpu, mem, 1), allocatable -= ... */
        const int32_t j = (int32_t)x[1];
        const int64_t dc = sign * x[2], dm = sign * x[3], dp = sign;
        if ((rcode = ksched_apply_delta(ctx, 1, &j, &dc, &dm, &dp)) != KSCHED_OK) die(ctx, "ksched_apply_delta", rcode);
    }
    int64_t *fc = malloc(8 * n), *fm = malloc(8 * n), *fp = malloc(8 * n);
    if ((rcode = ksched_read_nodes(ctx, n, fc, fm, fp)) != KSCHED_OK) die(ctx, "ksched_read_nodes", rcode);
    ksched_destroy(ctx);

    FILE *out = fopen(argv[2], "wb");
    if (!out) { perror("output"); return 1; }
    const int64_t stats[4] = {calls, binds, failed_binds, undone};
    fwrite(stats, 8, 4, out);
    fwrite(idx, 4, p, out);
    fwrite(score, 8, p, out);
    fwrite(feas, 4, p, out);
    fwrite(counts, 8, (size_t)p * KSCHED_NUM_REASONS, out);
    fwrite(fc, 8, n, out);
    fwrite(fm, 8, n, out);
    fwrite(fp, 8, n, out);
    fclose(out);
    printf("ksched_driver: %lld pods, %lld schedule calls, %lld binds, %lld failed binds, %lld commits undone\n",
           (long long)p, (long long)calls, (long long)binds, (long long)failed_binds, (long long)undone);
    return 0;
}
