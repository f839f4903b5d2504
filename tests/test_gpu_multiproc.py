"""GPU: the product multi-GPU entry point (model.model.sharded_infer) running the
library itself in two ranks.  The box has one GPU, so both ranks share cuda:0 and gather over
gloo; on a multi-GPU node the same code runs one rank per GPU over RCCL (infer.py / bench.py
under torchrun).  The ranks are fresh spawned interpreters; the single-process reference run
happens in another fresh process afterwards."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
N, B, T = 2112, 5, 4


def _paths():
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "speech-denoising-diffusion-model-2_amd"))


def _model():
    import torch
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from _helpers import UNET_NET, unet_params
    dev = torch.device("cuda", 0)
    net = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    m = M.SDDM(D.GaussianDiffusion("linear", T, 1e-6, 1e-3, device=dev), net, p_transition="condition_in")
    m.compute_dtype = "bfloat16"
    return m.to(dev)


def _rank(rank, world, port, out_path):
    _paths()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from model.model import sharded_infer
    from sddm_hip.synth import noisy_speech
    cond = torch.from_numpy(noisy_speech(B, N, seed=4321)).cuda()
    out = sharded_infer(_model(), cond, seed=13)
    if rank == 0:
        np.save(out_path, out.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def _single(rank, out_path):
    _paths()
    import torch
    from sddm_hip.synth import noisy_speech
    out = _model().infer(torch.from_numpy(noisy_speech(B, N, seed=4321)).cuda(), seed=13)
    np.save(out_path, out.cpu().numpy())


def test_two_ranks_on_the_library_equal_single_run(tmp_path):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    sharded, single = str(tmp_path / "sharded.npy"), str(tmp_path / "single.npy")
    mp.spawn(_rank, args=(2, port, sharded), nprocs=2, join=True)
    mp.spawn(_single, args=(single,), nprocs=1, join=True)
    a, b = np.load(sharded), np.load(single)
    assert a.shape == (B, 1, N) and np.isfinite(a).all()
    assert np.array_equal(a, b)


def _rccl_rank(rank, port, out_path):
    _paths()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)   # RCCL on ROCm
    assert dist.get_backend() == "nccl"
    from model.model import _all_gather_rows
    from sddm_hip.synth import noisy_speech
    seed = torch.tensor([13], dtype=torch.int64, device=dev)
    dist.broadcast(seed, src=0)                       # the seed hand-out of sharded_infer
    out = _model().infer(torch.from_numpy(noisy_speech(B, N, seed=4321)).cuda(), seed=int(seed.item()), row_offset=0)
    gathered = _all_gather_rows(out, None)            # all_gather_into_tensor on device buffers
    torch.cuda.synchronize()
    np.save(out_path, gathered.cpu().numpy())
    dist.destroy_process_group()


def test_rccl_collectives_of_the_sharded_path(tmp_path):
    """The RCCL (torch 'nccl' backend) calls of the multi-GPU path on the MI355X itself: a world-1
    group, sharded_infer's seed broadcast of a device tensor and _all_gather_rows'
    all_gather_into_tensor of the sampled rows; the gathered rows equal a single-process run bit
    for bit.  (RCCL refuses two ranks on one device; the 1/2/4/8-GPU curve is the driver's run.)"""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rccl, single = str(tmp_path / "rccl.npy"), str(tmp_path / "single.npy")
    mp.spawn(_rccl_rank, args=(port, rccl), nprocs=1, join=True)
    mp.spawn(_single, args=(single,), nprocs=1, join=True)
    a, b = np.load(rccl), np.load(single)
    assert a.shape == (B, 1, N) and np.isfinite(a).all()
    assert np.array_equal(a, b)
