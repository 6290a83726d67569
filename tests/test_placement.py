"""CPU tests of the GPU suite's rank placement (tests/gpu_workers.py rank_device): on a box with
several GPUs every rank gets its own (rank % ndev), as on the node, so `pytest -m gpu` is a
cross-device parity run there; on a 1-GPU box, or under MNCCL_TEST_COLOCATE=1, every rank shares
GPU 0 (the reference's perf_test topology, tests/perf_test.cpp:46)."""
import gpu_workers as GW


def test_one_rank_per_gpu_when_the_box_has_them():
    assert [GW.rank_device(r, 8, colocate=False) for r in range(8)] == list(range(8))
    assert [GW.ranks_sharing_device(r, 8, 8, colocate=False) for r in range(8)] == [1] * 8
    # more ranks than GPUs: dealt round robin (10 ranks on 8 GPUs: GPUs 0 and 1 hold two)
    assert [GW.rank_device(r, 8, colocate=False) for r in range(10)] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
    assert [GW.ranks_sharing_device(r, 10, 8, colocate=False) for r in range(10)] == [2, 2] + [1] * 6 + [2, 2]
    assert [GW.rank_device(r, 2, colocate=False) for r in range(3)] == [0, 1, 0]


def test_one_gpu_box_and_forced_colocation_share_gpu_0():
    assert [GW.rank_device(r, 1, colocate=False) for r in range(8)] == [0] * 8
    assert [GW.rank_device(r, 8, colocate=True) for r in range(8)] == [0] * 8
    assert GW.ranks_sharing_device(3, 8, 8, colocate=True) == 8
    assert GW.ranks_sharing_device(0, 3, 1, colocate=False) == 3


def test_colocate_switch_reads_the_environment(monkeypatch):
    monkeypatch.delenv("MNCCL_TEST_COLOCATE", raising=False)
    assert not GW.colocated() and GW.rank_device(5, 8) == 5
    monkeypatch.setenv("MNCCL_TEST_COLOCATE", "1")
    assert GW.colocated() and GW.rank_device(5, 8) == 0
    monkeypatch.setenv("MNCCL_TEST_COLOCATE", "0")
    assert not GW.colocated()
    assert GW.colocated({"MNCCL_TEST_COLOCATE": "1"}) and not GW.colocated({})
