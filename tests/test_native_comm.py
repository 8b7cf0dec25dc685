"""Native comm layer (csrc/comm, pcmx_comm.h): Cartesian topology, TCP transport, the native distributed
region growing (`bin/region`, counterpart of `mpirun -n P region pic1.bmp`) and the token chain
(`bin/mpi_ring`, counterpart of 1-introduction/mpi.c), launched by the native launcher `bin/pcmx_launch`
and by torchrun. GPU variants (RCCL transport) are marked gpu."""
import ctypes
import subprocess
import sys

import numpy as np
import pytest
from conftest import ASSETS, ROOT, cli_env

from parallel_c_programs_amd._native import cpu_lib
from parallel_c_programs_amd.parallel import CartTopology, dims_create, free_port
from parallel_c_programs_amd.utils import bmp

BIN = ROOT / "bin"


def _launch(n, *cmd, timeout=300):
    return subprocess.run([str(BIN / "pcmx_launch"), "-n", str(n), *map(str, cmd)], capture_output=True, text=True,
                          timeout=timeout, env=cli_env())


class Cart(ctypes.Structure):
    _fields_ = [("size", ctypes.c_int), ("dims", ctypes.c_int * 2)]


@pytest.mark.parametrize("n", list(range(1, 17)) + [24, 30, 64])
def test_native_dims_create_matches_python(n):
    d = (ctypes.c_int * 2)()
    cpu_lib().pcmx_dims_create(n, d)
    assert list(d) == dims_create(n)


def test_native_cart_tiles_match_python():
    lib = cpu_lib()
    for world in (1, 2, 3, 4, 6, 8):
        t = Cart()
        lib.pcmx_cart_init(ctypes.byref(t), world, None)
        topo = CartTopology.create(world)
        for r in range(world):
            out = (ctypes.c_int * 4)()
            lib.pcmx_cart_tile(ctypes.byref(t), r, 512, 300, out)
            assert tuple(out) == topo.tile(r, 512, 300)
            nb = (ctypes.c_int * 4)()
            lib.pcmx_cart_neighbours(ctypes.byref(t), r, nb)
            py = topo.neighbours(r)
            assert list(nb) == [py["north"], py["south"], py["west"], py["east"]]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_native_region_tcp_golden(tmp_path, n):
    r = _launch(n, BIN / "region", "--cpu", ASSETS / "pic1.bmp")
    assert r.returncode == 0, r.stderr
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


def test_native_region_explicit_dims_and_other_image(tmp_path):
    from parallel_c_programs_amd import ops
    import torch

    r = _launch(6, BIN / "region", "--cpu", "--dims", 2, 3, ASSETS / "pic3.bmp")
    assert r.returncode == 0, r.stderr
    img = torch.from_numpy(bmp.read(ASSETS / "pic3.bmp"))
    want = ops.apply_region_mask(img, ops.region2d(img)).numpy()
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), want)


def test_native_region_usage():
    r = subprocess.run([str(BIN / "region")], capture_output=True, text=True, env=cli_env())
    assert r.stdout == "Useage: region file" and r.returncode == 255


def test_native_mpi_ring_tcp():
    r = _launch(4, BIN / "mpi_ring", "--cpu")
    assert r.returncode == 0, r.stderr
    lines = set(r.stdout.splitlines())
    assert "Rank 0 received 5 " in lines and "Rank 3 received 2 " in lines and "Rank 3 sent 3 " in lines


def test_native_region_under_torchrun(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "--no-python", str(BIN / "region"), "--cpu",
           str(ASSETS / "pic1.bmp")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=cli_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


def test_launcher_propagates_failure():
    r = _launch(3, "sh", "-c", 'test "$RANK" != 1')
    assert r.returncode == 1


@pytest.mark.gpu
def test_native_region_rccl_golden(gpu, tmp_path):
    r = _launch(1, BIN / "region", ASSETS / "pic1.bmp")
    assert r.returncode == 0, r.stderr
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


@pytest.mark.gpu
def test_native_mpi_ring_rccl_single_rank(gpu):
    r = _launch(1, BIN / "mpi_ring")
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_native_region_multirank_one_gpu_staged(gpu, tmp_path, n):
    """P ranks share the single GPU: gfx950 tile kernels + device pack/unpack + grouped exchange schedule,
    with halos staged over TCP (RCCL refuses two ranks per device)."""
    r = _launch(n, BIN / "region", "--staged", ASSETS / "pic1.bmp")
    assert r.returncode == 0, r.stderr
    assert np.array_equal(bmp.read(tmp_path / "out.bmp"), bmp.read(ASSETS / "region_pic1_golden.bmp"))


@pytest.mark.gpu
def test_native_mpi_ring_staged(gpu):
    r = _launch(3, BIN / "mpi_ring", "--staged")
    assert r.returncode == 0, r.stderr
    assert "Rank 0 received 3 " in r.stdout.splitlines()


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_native_collectives_tcp(n):
    """MPI_Allgather / Gather / Scatter / Alltoall equivalents (pcmx_comm_allgather ...) over the TCP transport:
    every rank checks its blocks byte for byte (odd block size, in-place all-gather, non-zero gather root)."""
    r = _launch(n, BIN / "collectives", "--cpu", "--bytes", "4099")
    assert r.returncode == 0, r.stderr
    assert f"collectives ok world={n}" in r.stdout
    assert sum("alltoall ok" in ln for ln in r.stdout.splitlines()) == n


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_native_collectives_staged(gpu, n):
    """Device buffers, P ranks on the one GPU: the collectives plus the distributed reduce and prefix scan
    (local gfx950 reduce/scan kernels, per-rank totals all-gathered, exact on small integers, ragged ranks)."""
    r = _launch(n, BIN / "collectives", "--staged")
    assert r.returncode == 0, r.stderr
    assert f"collectives ok world={n}" in r.stdout
    assert sum("reduce scan ok" in ln for ln in r.stdout.splitlines()) == n


@pytest.mark.gpu
def test_native_collectives_rccl(gpu):
    import torch

    n = min(torch.cuda.device_count(), 8)
    r = _launch(n, BIN / "collectives")
    assert r.returncode == 0, r.stderr
    assert f"collectives ok world={n}" in r.stdout


def test_tcp_transport_error_codes_world1():
    """TCP transport failures reach the caller as the shared PCMX_ERR_* codes (pcmx_errors.h): a peer out of range
    and a send/recv-to-self size mismatch are argument errors (-1), not timeouts or allocation failures."""
    import ctypes

    from parallel_c_programs_amd._native import cpu_lib
    from parallel_c_programs_amd.parallel import free_port

    lib = cpu_lib()
    comm = ctypes.c_void_p()
    assert lib.pcmx_comm_init_tcp(0, 1, b"127.0.0.1", free_port(), ctypes.byref(comm)) == 0
    try:
        a, b = ctypes.create_string_buffer(16), ctypes.create_string_buffer(16)
        assert lib.pcmx_comm_send(comm, a, ctypes.c_size_t(4), 3) == -1  # peer 3 of world 1
        assert lib.pcmx_comm_group_start(comm) == 0
        assert lib.pcmx_comm_send(comm, a, ctypes.c_size_t(8), 0) == 0
        assert lib.pcmx_comm_recv(comm, b, ctypes.c_size_t(4), 0) == 0
        assert lib.pcmx_comm_group_end(comm) == -1  # size mismatch of the self pair
        assert lib.pcmx_comm_group_end(comm) == -1  # no group open
        a.value = b"abcdefg"
        assert lib.pcmx_comm_group_start(comm) == 0
        assert lib.pcmx_comm_send(comm, a, ctypes.c_size_t(8), 0) == 0
        assert lib.pcmx_comm_recv(comm, b, ctypes.c_size_t(8), 0) == 0
        assert lib.pcmx_comm_group_end(comm) == 0 and b.value == b"abcdefg"
    finally:
        lib.pcmx_comm_destroy(comm)
