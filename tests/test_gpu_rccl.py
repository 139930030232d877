"""RCCL on the real GPU: a 1-rank ``nccl`` (= RCCL on ROCm) process group gathers the worker's
letterboxed consumer batch with ``all_gather_into_tensor`` — the same collective the 8-GPU
camera-DP path uses (bench.py, parallel.ConsumerBatch) — so the RCCL path runs on every GPU
test round even on a 1-GPU box. Multi-rank correctness is covered with gloo on CPU
(tests/test_parallel.py)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_group():
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)


def test_consumer_batch_rccl_allgather(nccl_group):
    from video_edge_ai_proxy_amd import native
    from video_edge_ai_proxy_amd.parallel import ConsumerBatch

    dist = nccl_group
    dev = torch.device("cuda", 0)
    w = native.Worker(device=0, letterbox_size=64, max_cameras=3, letterbox_format=0)
    cb = ConsumerBatch(w, 3, 64, dev, world=1)
    assert cb.collective
    cfg = native.SynthConfig()
    cfg.width, cfg.height, cfg.gop = 160, 96, 4
    cfg.compressed = True
    rb = native.ReplayBench(w, 3, cfg, cached_frames=4, threads=2, prefix="rccl")
    for _ in range(4):
        cb.prepare()
        rb.step()
        out, work = cb.gather(async_op=True)
        work.wait()
    cb.drain()
    torch.cuda.synchronize()
    local = cb.bufs[(cb.tick - 1) & 1]
    assert out.shape == (3, 64, 64, 3) and out.is_cuda
    assert torch.equal(out, local)
    assert int(local.float().sum().item()) > 0  # letterbox wrote frames
    # the camera rows differ (different seeds): the gather did not replicate one row
    assert not torch.equal(local[0], local[1])
    # and a reduction over the same communicator
    t = torch.arange(8, device=dev, dtype=torch.float32)
    dist.all_reduce(t)
    assert torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32))
