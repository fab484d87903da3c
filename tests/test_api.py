"""MPI-style API: coverage of every reference wrapper name and
multi-process behaviour (CPU here; HBM buffers on the GPU box)."""
import re

import pytest

from mp_util import ROOT, run_ranks

CHECKS = ["ring_send_recv", "large_message", "probe_any_source", "message_ordering", "cancel_recv", "ssend",
          "sendrecv_persistent", "facade_count_datatype", "allreduce_iallreduce", "reductions", "collectives", "groups_comms", "topologies",
          "datatypes", "windows", "mpi_io", "intercomm", "mpiT_api", "objects"]


def test_every_reference_wrapper_has_a_counterpart():
    import os

    import mpit_amd.mpiT as M

    survey = open(os.path.join(ROOT, "SURVEY.md")).read()
    names = set(re.findall(r"`([A-Z][A-Za-z_]+):\d+`", survey))
    assert len(names) >= 250, len(names)
    dropped = {"Comm_create_errhandler", "Comm_spawn", "Comm_spawn_multiple", "File_create_errhandler",
               "Group_range_excl", "Group_range_incl", "Init", "Init_thread", "Op_commutative", "Pcontrol",
               "Reduce_local", "Win_create_errhandler", "Init_MTF", "Init_MTS", "Init_MTM"}
    missing = sorted(n for n in names | dropped if not hasattr(M, n))
    assert not missing, missing
    for c in ["CHAR", "BYTE", "SHORT", "INT", "LONG", "FLOAT", "DOUBLE", "UNSIGNED_CHAR", "UNSIGNED_SHORT",
              "UNSIGNED", "UNSIGNED_LONG", "LONG_DOUBLE", "LONG_LONG_INT", "FLOAT_INT", "LONG_INT", "DOUBLE_INT",
              "SHORT_INT", "2INT", "LONG_DOUBLE_INT", "PACKED", "UB", "LB", "ANY_SOURCE", "PROC_NULL", "ROOT",
              "ANY_TAG", "UNDEFINED", "CART", "GRAPH", "KEYVAL_INVALID", "MAX", "MIN", "SUM", "PROD", "LAND", "BAND",
              "LOR", "BOR", "LXOR", "BXOR", "MINLOC", "MAXLOC", "IDENT", "CONGRUENT", "SIMILAR", "UNEQUAL",
              "SUCCESS", "ERR_TRUNCATE", "ERR_LASTCODE", "GROUP_EMPTY", "signal_INIT", "signal_DONE",
              "tag_ps_recv_init", "tag_ps_recv_grad_tail"]:
        assert hasattr(M, c), c


@pytest.mark.parametrize("n", [2, 3, 4])
def test_api_suite_cpu(n):
    out = run_ranks("api_suite.py", n, {"MPIT_CPU_ONLY": "1"}, timeout=300)
    for c in CHECKS:
        assert f"OK {c}" in out, (c, out[-3000:])
    assert "ALL_DONE" in out


@pytest.mark.parametrize("n", [2, 3])
def test_api_suite_cpu_torch_distributed_branch(n):
    """Every host collective through torch.distributed (gloo) instead of the shm
    point-to-point algorithms: the branch HBM tensors take with RCCL on a multi-GPU node —
    Iallreduce's Request(work=...), all_gather_into_tensor, all_to_all_single,
    reduce_scatter_tensor, broadcast / reduce — runs here at least once; sub-communicators
    stay on the point-to-point engine (comm.py Comm._use_rccl)."""
    out = run_ranks("api_suite.py", n, {"MPIT_CPU_ONLY": "1", "MPIT_DIST_HOST": "1"}, timeout=300)
    for c in CHECKS:
        assert f"OK {c}" in out, (c, out[-3000:])
    assert "ALL_DONE" in out
    assert "DIST_WORK_REQUEST" in out


@pytest.mark.gpu
def test_api_suite_gpu_two_ranks_one_device():
    out = run_ranks("api_suite.py", 2, {"T_DEVICE": "cuda"}, timeout=300)
    for c in CHECKS:
        assert f"OK {c}" in out, (c, out[-3000:])


@pytest.mark.gpu
def test_api_suite_gpu_three_ranks_one_device():
    """HBM tensors with n > 2 ranks sharing a GPU take the point-to-point ring
    all-reduce (RCCL cannot put two ranks on one device); its chunk updates read the receive
    buffer asynchronously, so the ring alternates two of them (comm.py _ring_allreduce)."""
    out = run_ranks("api_suite.py", 3, {"T_DEVICE": "cuda"}, timeout=300)
    for c in CHECKS:
        assert f"OK {c}" in out, (c, out[-3000:])
