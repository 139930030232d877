"""bench.py --source records (the GPU-side ceiling): ReplayBench(records=True) parses every
camera's looped GOPs once up front and replays the reconstruction jobs with no host parse in the
timed loop. The replayed jobs must still publish exactly the frames a decoder produces for the
looped stream (checked against the CPU reference decoder, by pts), on the CPU backend and on
gfx950 (the same records, gathered over PCIe into the GPU lanes)."""
import numpy as np
import pytest

from conftest import synth


@pytest.mark.parametrize("device", [-1, pytest.param(0, marks=pytest.mark.gpu)])
def test_records_replay_publishes_decoder_frames(native, device):
    c = native.SynthConfig()
    c.width, c.height, c.gop, c.fps, c.seed = 320, 192, 10, 30, 5
    c.compressed, c.profile, c.bframes, c.cabac = True, "high", 2, True
    c.temporal_noise = 1.0
    # the camera-0 stream ReplayBench encodes (seed and IDR phase of camera 0 = the config's)
    enc = native.SynthH264(c)
    aus = [enc.next() for _ in range(c.gop * 2)]
    ref, dec = {}, native.CpuDecoder()
    for a in aus + aus:  # two cycles: the second one's outputs are the steady state
        img = dec.decode(a)
        if img is not None:
            ref[dec.last_pts] = img
    w = native.Worker(device=device, max_cameras=2)
    rb = native.ReplayBench(w, 1, c, cached_frames=c.gop * 2, threads=1, records=True, prefix="rec")
    cam = list(rb.cameras)[0]
    seq, checked = 0, 0
    for _ in range(3 * c.gop * 2):  # three replay cycles
        rb.step()
        rb.drain()
        r = w.read_latest(cam, seq)
        if r is None:
            continue
        meta, img = r
        seq = meta["seq"]
        want = ref[meta["pts"]]
        assert np.array_equal(img, want), f"pts {meta['pts']}: {int((img != want).sum())} samples differ"
        checked += 1
    assert checked >= 3 * c.gop * 2 - 4 and rb.parse_failures == 0
    assert w.pictures >= 3 * c.gop * 2
