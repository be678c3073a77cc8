"""The persistent pipeline's failure path: every wait is bounded, a timeout ends
every role of the kernel and names where the workgroups stood, and the context stays usable -- the next call
(persistent, or the stream pipeline) is bit-exact against the oracle again.

The timeout is forced with ksched_set_timeout(ctx, 0): every wait not satisfied by its first poll gives up.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_persistent_timeout_reports_and_recovers(gpu_available, oracle_mod):
    from ksched import MODE_BATCHED, Engine, KschedError, cluster
    cl = cluster.make_cluster("c3", n_nodes=20000, n_pods=3000)
    want = oracle_mod.schedule(cl, nthreads=8)
    with Engine(mode=MODE_BATCHED, priority=cl.priority, domain=cl.domain, use_labels=cl.use_labels,
                topk=16, batch=64) as e:
        e.load_nodes(cl.alloc_cpu, cl.alloc_mem, cl.alloc_pods, labels=cl.labels, price=cl.price)
        e.save_state()
        e.upload_pods(cl.req_cpu, cl.req_mem, cl.req_pods, cl.selector)

        e.set_timeout(0)
        with pytest.raises(KschedError) as ex:
            e.run()
            e.sync()
        msg = str(ex.value)
        assert "persistent pipeline" in msg and "timed out" in msg, msg
        # the progress words: the score workgroups' batches and both commit workgroups' batch and phase
        assert "score batches" in msg and "commit workgroup 0" in msg and "commit workgroup 1" in msg, msg
        e.set_timeout(10000)

        def again():
            e.restore_state()
            e.run()
            e.sync()
            oi, os_, of = e.results()
            assert np.array_equal(oi, want[0])
            assert np.array_equal(os_.view(np.int64), want[1].view(np.int64))
            assert np.array_equal(of, want[2])
            return e.stats()["pipeline"]

        assert again() == "persistent"
        assert again() == "persistent"
