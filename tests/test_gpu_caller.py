"""Caller-side HIP kernels against the reference's own outputs (tests/golden/caller_utils.npz,
written by tests/golden/make_golden.py from core/utils/utils.py): replicate padding (exact),
forward_interpolate (exact: the same nearest source), bilinear_sampler (1e-6) + its mask,
and the batched .flo writer."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_input_padder_gpu_matches_reference():
    from raft_optical_flow_amd import InputPadder
    g = load_golden("caller_utils.npz")
    x = torch.from_numpy(g["pad_in"]).to(DEV)
    for mode, key in (("sintel", "pad_sintel"), ("kitti", "pad_kitti")):
        p = InputPadder(x.shape, mode=mode)
        y, = p.pad(x)
        assert y.is_cuda and np.array_equal(y.cpu().numpy(), g[key])
        assert torch.equal(p.unpad(y), x)


def test_input_padder_cpu_tensor_round_trips_through_gpu():
    from raft_optical_flow_amd import InputPadder
    g = load_golden("caller_utils.npz")
    x = torch.from_numpy(g["pad_in"])
    y, = InputPadder(x.shape).pad(x)
    assert not y.is_cuda and np.array_equal(y.numpy(), g["pad_sintel"])


@pytest.mark.parametrize("name", ["fi_smooth", "fi_leaving", "fi_zero"])
def test_forward_interpolate_matches_reference(name):
    from raft_optical_flow_amd.utils.utils import forward_interpolate
    g = load_golden("caller_utils.npz")
    f = torch.from_numpy(g[name + "_in"]).to(DEV)
    out = forward_interpolate(f)
    assert out.is_cuda and out.shape == f.shape
    assert np.array_equal(out.cpu().numpy(), g[name + "_out"])
    # batched form
    out2 = forward_interpolate(torch.stack([f, f]))
    assert torch.equal(out2[1], out)


def test_bilinear_sampler_matches_reference():
    from raft_optical_flow_amd.utils.utils import bilinear_sampler
    g = load_golden("caller_utils.npz")
    out, m = bilinear_sampler(torch.from_numpy(g["bs_img"]).to(DEV), torch.from_numpy(g["bs_coords"]).to(DEV),
                              mask=True)
    assert float(np.abs(out.cpu().numpy() - g["bs_out"]).max()) < 1e-6
    assert np.array_equal(m.cpu().numpy(), g["bs_mask"])


def test_write_flo_batch(tmp_path):
    from raft_optical_flow_amd import io as rio
    flows = torch.randn(3, 2, 9, 13, device=DEV)
    paths = [str(tmp_path / f"f{i}.flo") for i in range(3)]
    rio.write_flo_batch(paths, flows)
    for i in range(3):
        assert np.array_equal(rio.readFlow(paths[i]), flows[i].permute(1, 2, 0).cpu().numpy())
