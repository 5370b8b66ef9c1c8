"""Single-process multi-device frames (sdf_render_multi, sdf3d_amd/csrc/multi.cpp;
SURVEY.md 8(b)): the frame assembled from the root's own rows and the other
devices' TILES streams, decoded through peer-mapped memory, equals a
one-device sdf_render bit for bit.  One GPU here, so the device list repeats
device 0: every share still goes the multi-device way (TILES render and
compaction on its own stream and buffer set, cross-stream events, in-place
decode through a per-part pointer)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _whole(rd, f):
    ref, _ = rd.render(f)
    torch.cuda.synchronize()
    return ref


@pytest.mark.parametrize("ndev,cfg,W,H,shares", [
    (1, "C3", 320, 180, (0, 0)), (2, "C3", 320, 183, (0, 0)), (3, "C3", 200, 120, (1, 2)),
    (8, "C3", 480, 270, (0, 0)), (8, "C4", 3840, 2160, (0, 0)), (4, "C5", 256, 144, (3, 4)),
    (8, "REF", 37, 23, (1, 1))])
def test_render_multi_matches_single_device(ndev, cfg, W, H, shares):
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(cfg, W, H, precision=abi.PRECISION_FAST, pose=1)
    got = rd.render_multi(f, [0] * ndev, shares=shares)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), _whole(rd, f).view(torch.int32))


def test_render_multi_frame_sequence():
    """Successive frames on one stream alternate the two buffer sets; a
    camera change per frame lands in exactly its frame."""
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    s = torch.cuda.Stream()
    outs, frames = [], []
    for i in range(5):
        f = scenes.config("C3", 256, 144, precision=abi.PRECISION_FAST, pose=i % 4)
        frames.append(f)
        outs.append(rd.render_multi(f, [0, 0, 0, 0], stream=s))
    s.synchronize()
    for f, o in zip(frames, outs):
        assert torch.equal(o.view(torch.int32), _whole(rd, f).view(torch.int32))


def test_render_multi_rejects_bad_arguments():
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    f = scenes.config("C3", 64, 32, precision=abi.PRECISION_FAST)
    g = f.copy()
    g.params.output_format = abi.FORMAT_RGBA8
    with pytest.raises(abi.SdfError):
        rd.render_multi(g, [0, 0], out=torch.empty((32, 64, 4), device="cuda:0"))
    with pytest.raises(abi.SdfError):
        rd.render_multi(f, [0, 99])          # no such device
    with pytest.raises(ValueError):
        rd.render_multi(f, [1, 0])           # devices[0] must be the renderer's
    # a refused call leaves no stale HIP error behind for the next launch
    rd.render(f)
    torch.cuda.synchronize()
    abi.load_library().sdf_render_multi_release()
