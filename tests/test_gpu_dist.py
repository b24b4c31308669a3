"""The d-slice path on the GPU: slice keys from the HIP kernel, the MIN reduction
(reduce-scatter + uint8 all-gather, or all-reduce) and the device key -> disparity conversion,
against the single-GPU full-range match.  Ranks: one RCCL rank, and two gloo ranks sharing the
one GPU (gloo collectives are staged through host copies; the kernels and the chunking are the
ones an 8-GPU RCCL run uses)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pair(W, H, D):
    from oracle import oracle as O
    return O.synth_pair(777, W, H, D)


@pytest.mark.parametrize("coll", ["rs_ag", "allreduce"])
def test_dslice_one_rccl_rank(coll):
    import torch
    import torch.distributed as dist
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import sharding
    W, H, D, r = 333, 121, 256, 5
    L, R = _pair(W, H, 64)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        with sm.BlockMatcher(0, 512, 256, 256) as m:
            Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
            got = sharding.match_dslice(m, Lt, Rt, r, D, 0, 1, collective=coll)
            want = m.match_device(Lt, Rt, r, D)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), want.cpu().numpy())
    finally:
        dist.destroy_process_group()


def _worker(rank, world, port, coll, W, H, D, r, out_dir):
    import torch
    import torch.distributed as dist
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L, R = _pair(W, H, 64)
    with sm.BlockMatcher(0, 512, 256, 256) as m:
        Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        got = sharding.match_dslice(m, Lt, Rt, r, D, rank, world, collective=coll)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"d{rank}.npy"), got.cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("coll,world", [("rs_ag", 2), ("allreduce", 2), ("rs_ag", 3)])
def test_dslice_gloo_ranks_share_gpu(tmp_path, coll, world):
    import torch.multiprocessing as mp
    from oracle import oracle as O
    W, H, D, r = 301, 67, 200, 4        # W*H = 20167: padded to the world size for the reduce-scatter
    mp.spawn(_worker, args=(world, _free_port(), coll, W, H, D, r, str(tmp_path)), nprocs=world, join=True)
    L, R = _pair(W, H, 64)
    want = O.box_disp(L, R, r, D)
    for k in range(world):
        assert np.array_equal(np.load(tmp_path / f"d{k}.npy"), want)
