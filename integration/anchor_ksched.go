// anchor_ksched.go -- the cgo shim a maintainer drops into the reference's `anchor` package
// (package main, next to anchor/schedule.go) to run predicate + priorities on libksched.
//
// It replaces the bodies of schedulePods (anchor/schedule.go:185-197, the reconcile loop's batch driver:
// schedulePodsGPU below) and of schedulePod (anchor/schedule.go:68-89, what monitorUnscheduledPods calls for
// every watched ADDED pod, anchor/schedule.go:47-66: schedulePodGPU below): the predicate / priorities
// evaluation of every pod against every node (anchor/predicate.go:107-176, anchor/priorities.go:25-63) and the
// "next pod sees the previous bind" accounting (usedResource, anchor/predicate.go:83-105) run on the
// GPU; getNodes/getPods (anchor/tools.go:53-108), bind and postEvent (anchor/schedule.go:200-261,
// anchor/tools.go:22-51) are the reference's own functions, called unchanged and in pod order.  The two call
// sites change by one identifier each: schedulePods() -> schedulePodsGPU() in reconcileUnscheduledPods
// (anchor/schedule.go:37) and schedulePod(&pod) -> schedulePodGPU(&pod) in monitorUnscheduledPods (:57).
//
// This file is not compiled in this repository's image (no Go toolchain); the same call sequences --
// create, load_nodes, schedule, explain_pod per NO_FIT pod, ordered binds, apply_delta undo of a failed
// bind, for a whole pending list and for one watched pod at a time -- are compiled and run against
// libksched.so as integration/ksched_driver.c (batch and watch modes) by tests/test_gpu_integration.py.  Type-checked by
// inspection against the reference: NodeList.Items is
// []*Node (anchor/types.go:99), getUnscheduledPods returns []*Pod (anchor/schedule.go:145),
// allocatableResource / bind take *Node (anchor/predicate.go:56, anchor/schedule.go:200),
// usedResource takes (*NodeList, *PodList) (anchor/predicate.go:83), requestedResource *Pod
// (anchor/predicate.go:69), postEvent an Event (anchor/tools.go:22, anchor/types.go:4-40).
// Build (with the reference checked out beside this repository):
//
//	CGO_CFLAGS=-I<repo>/include CGO_LDFLAGS="-L<repo>/k8s-scheduler_amd -lksched" go build -o scheduler anchor/*.go
package main

/*
#cgo LDFLAGS: -lksched
#include <stdlib.h>
#include "ksched.h"
*/
import "C"

import (
	"fmt"
	"log"
	"strings"
	"time"
	"unsafe"
)

var kctx *C.ksched_ctx

// kschedInit creates the engine once at startup (main.go:24-50 would call it before the loops start).
func kschedInit() {
	var o C.ksched_opts
	C.ksched_default_opts(&o)
	o.mode = C.KSCHED_MODE_AUTO            // one pod: exact persistent kernel; many: batched
	o.priority = C.KSCHED_PRIORITY_RESOURCE // (balanced + least requested) / 2, anchor/priorities.go:45-50
	o.domain = C.KSCHED_DOMAIN_ALL          // the reference's argmax ranges over every node
	if rc := C.ksched_create(&o, &kctx); rc != C.KSCHED_OK {
		log.Fatalf("ksched_create failed: %d", int(rc))
	}
}

func kschedCheck(rc C.int, what string) {
	if rc != C.KSCHED_OK {
		// the reference's errFatal convention for unrecoverable failures (anchor/tools.go:110-115)
		log.Fatalf("%s failed (%d): %s", what, int(rc), C.GoString(C.ksched_last_error(kctx)))
	}
}

func i64p(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}

// loadCluster packs the API server's view exactly as predicate() does per pod -- allocatable =
// capacity - used (anchor/predicate.go:56-67, 83-105) -- and makes it the device's node state.
func loadCluster(nodeList *NodeList, podList *PodList) {
	used := usedResource(nodeList, podList)
	n := len(nodeList.Items)
	ac, am, ap := make([]int64, n), make([]int64, n), make([]int64, n)
	for i := range nodeList.Items {
		a := allocatableResource(nodeList.Items[i], used) // Items is []*Node (anchor/types.go:99); takes *Node (anchor/predicate.go:56)
		ac[i], am[i], ap[i] = a.CPU, a.Memory, a.Pod
	}
	kschedCheck(C.ksched_load_nodes(kctx, C.int64_t(n), i64p(ac), i64p(am), i64p(ap), nil, nil), "ksched_load_nodes")
}

// failedSchedulingEvent posts predicate()'s FailedScheduling event (anchor/predicate.go:152-173) for
// pods[i], pod i of the last ksched_schedule call, with the failures list of the state it saw.
func failedSchedulingEvent(pod *Pod, i int, nodeList *NodeList) {
	var counts [C.KSCHED_NUM_REASONS]C.int64_t
	reason := make([]uint8, len(nodeList.Items))
	var rp *C.uint8_t // out_reason may be NULL: an empty node list has no per-node lines
	if len(reason) > 0 {
		rp = (*C.uint8_t)(unsafe.Pointer(&reason[0]))
	}
	kschedCheck(C.ksched_explain_pod(kctx, C.int64_t(i), &counts[0], rp), "ksched_explain_pod")
	text := map[uint8]string{C.KSCHED_REASON_CPU: "Insufficient CPU",
		C.KSCHED_REASON_MEMORY: "Insufficient Memory", C.KSCHED_REASON_POD: "Insufficient Pod"}
	failures := make([]string, 0, len(reason))
	for j, node := range nodeList.Items {
		if reason[j] != C.KSCHED_REASON_FIT {
			failures = append(failures, fmt.Sprintf("fit failure on node (%s): %s", node.Metadata.Name, text[reason[j]]))
		}
	}
	timestamp := time.Now().UTC().Format(time.RFC3339)
	postEvent(Event{
		Count:          1,
		Message:        fmt.Sprintf("pod (%s) failed to fit in any node\n%s", pod.Metadata.Name, strings.Join(failures, "\n")),
		Metadata:       Metadata{GenerateName: pod.Metadata.Name + "-"},
		Reason:         "FailedScheduling",
		LastTimestamp:  timestamp,
		FirstTimestamp: timestamp,
		Type:           "Warning",
		Source:         EventSource{Component: "hightower-scheduler"},
		InvolvedObject: ObjectReference{Kind: "Pod", Name: pod.Metadata.Name, Namespace: "default", Uid: pod.Metadata.Uid},
	})
}

// schedulePodsGPU is schedulePods (anchor/schedule.go:185-197) on the engine: one call resolves every
// pending pod in order, then the binds follow in the same order.  A failed bind leaves its pod
// unbound, and in the reference every later pod re-reads a cluster without it, so the commits of that
// pod and of every later placement of the call (none of them bound yet) are undone and the pods after
// it are scheduled again.
func schedulePodsGPU() error {
	processorLock.Lock()
	defer processorLock.Unlock()
	pods, err := getUnscheduledPods()
	if err != nil {
		return err
	}
	nodeList, err := getNodes()
	errFatal(err, "failed to get nodes")
	podList, err := getPods()
	errFatal(err, "failed to get pods")
	loadCluster(nodeList, podList)

	p := len(pods)
	rc, rm, rp := make([]int64, p), make([]int64, p), make([]int64, p)
	for i, pod := range pods {
		r := requestedResource(pod) // anchor/predicate.go:69-81 (Pod = #containers)
		rc[i], rm[i], rp[i] = r.CPU, r.Memory, r.Pod
	}
	idx := make([]int32, p)
	for start := 0; start < p; {
		m := p - start
		kschedCheck(C.ksched_schedule(kctx, C.int64_t(m), i64p(rc[start:]), i64p(rm[start:]), i64p(rp[start:]), nil,
			(*C.int32_t)(unsafe.Pointer(&idx[start])), nil, nil), "ksched_schedule")
		resume := -1
		for i := start; i < p && resume < 0; i++ {
			pod := pods[i]
			switch idx[i] {
			case C.KSCHED_NO_FIT: // predicate() found no node (anchor/schedule.go:74-76)
				failedSchedulingEvent(pod, i-start, nodeList)
				errPrintln(fmt.Errorf("Unable to schedule pod (%s) failed to fit in any node", pod.Metadata.Name),
					"pod schedule failed")
			case C.KSCHED_NO_POSITIVE_SCORE: // the reference binds a nil node here and panics
				errPrintln(fmt.Errorf("no node scored > 0 for pod (%s)", pod.Metadata.Name), "pod schedule failed")
			default:
				err := bind(pod, nodeList.Items[idx[i]]) // unchanged HTTP bind; Items[k] is *Node (anchor/schedule.go:200)
				if err != nil {
					errPrintln(err, "pod schedule failed")
					var ui []int32
					var dc, dm, dp []int64
					for j := i; j < p; j++ {
						if idx[j] >= 0 {
							ui = append(ui, idx[j])
							dc, dm, dp = append(dc, rc[j]), append(dm, rm[j]), append(dp, 1)
						}
					}
					var uip *C.int32_t // never empty here (pod i itself was placed), guarded all the same
					if len(ui) > 0 {
						uip = (*C.int32_t)(unsafe.Pointer(&ui[0]))
					}
					kschedCheck(C.ksched_apply_delta(kctx, C.int64_t(len(ui)), uip, i64p(dc), i64p(dm), i64p(dp)),
						"ksched_apply_delta")
					resume = i + 1
				}
			}
		}
		if resume < 0 {
			break
		}
		start = resume
	}
	return nil
}

// schedulePodGPU is schedulePod (anchor/schedule.go:68-89) on the engine, for monitorUnscheduledPods
// (anchor/schedule.go:47-66, which holds processorLock around the call).  predicate() re-reads the nodes and every
// pod per call and recounts usedResource (anchor/predicate.go:107-115), so the cluster is loaded again here; then
// the one pod is scheduled on the device (KSCHED_MODE_AUTO: the exact kernel for a single pod).  No node fits:
// predicate()'s FailedScheduling event (failedSchedulingEvent, from ksched_explain_pod) and the reference's error.
// A placement is bound with the reference's bind, unchanged; a failed bind returns its error, and the engine's
// commit of the pod is undone so that its state is the API server's again.
func schedulePodGPU(pod *Pod) error {
	nodeList, err := getNodes()
	errFatal(err, "failed to get nodes")
	podList, err := getPods()
	errFatal(err, "failed to get pods")
	loadCluster(nodeList, podList)

	r := requestedResource(pod) // anchor/predicate.go:69-81 (Pod = #containers)
	rc, rm, rp := []int64{r.CPU}, []int64{r.Memory}, []int64{r.Pod}
	var idx C.int32_t
	kschedCheck(C.ksched_schedule(kctx, 1, i64p(rc), i64p(rm), i64p(rp), nil, &idx, nil, nil), "ksched_schedule")
	switch idx {
	case C.KSCHED_NO_FIT: // predicate() returned no node (anchor/schedule.go:74-76), after posting its event
		failedSchedulingEvent(pod, 0, nodeList)
		return fmt.Errorf("Unable to schedule pod (%s) failed to fit in any node", pod.Metadata.Name)
	case C.KSCHED_NO_POSITIVE_SCORE: // the reference binds a nil node here and panics
		return fmt.Errorf("no node scored > 0 for pod (%s)", pod.Metadata.Name)
	}
	if err := bind(pod, nodeList.Items[idx]); err != nil { // unchanged HTTP bind (anchor/schedule.go:200)
		one := []int64{1}
		kschedCheck(C.ksched_apply_delta(kctx, 1, &idx, i64p(rc), i64p(rm), i64p(one)), "ksched_apply_delta")
		return err
	}
	return nil
}
