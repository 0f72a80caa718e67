"""Host-side API parity that needs no GPU: module trees / state_dict keys, checkpoint
loading (raft-small.pth contents, DataParallel `module.` prefix), argparse quirks,
InputPadder, the compat shims, and loud failure without a GPU."""
import argparse
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, load_golden
from oracle import raft_oracle as O
from raft_optical_flow_amd import RAFT, InputPadder
from raft_optical_flow_amd.init import seeded_state_dict


def ns(**kw):
    return argparse.Namespace(**kw)


def test_state_dict_key_counts_match_reference():
    # survey: 179 tensors for RAFT-full (incl. 45 BN buffers), 106 for RAFT-small
    full = RAFT(ns(small=False, mixed_precision=False))
    small = RAFT(ns(small=True, mixed_precision=False))
    assert len(full.state_dict()) == 179
    assert len(small.state_dict()) == 106
    assert sum(p.numel() for p in full.parameters()) == 5_257_536
    assert sum(p.numel() for p in small.parameters()) == 990_162


def test_raft_small_checkpoint_loads_strict_with_dataparallel_prefix():
    wts = load_golden("raft_small_weights.npz")
    m = torch.nn.DataParallel(RAFT(ns(small=True, mixed_precision=False)))
    m.load_state_dict({"module." + k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)


def test_args_defaults_written_back_like_reference():
    a = ns(small=False, mixed_precision=False)
    RAFT(a)
    assert a.corr_levels == 4 and a.corr_radius == 4 and a.dropout == 0 and a.alternate_corr is False
    a = ns(small="yes", mixed_precision=False)  # --small default=True, any string is truthy
    m = RAFT(a)
    assert a.corr_radius == 3 and m.hidden_dim == 96


def test_input_padder_pads():
    p = InputPadder((1, 3, 436, 1024))
    assert p._pad == [0, 0, 2, 2] and p._pad == O.InputPadder((1, 3, 436, 1024))._pad
    assert InputPadder((1, 3, 540, 960), mode="kitti")._pad == [0, 0, 0, 4]
    x = torch.zeros(1, 3, 440, 1024)
    assert p.unpad(x).shape[-2:] == (436, 1024)


def test_forward_fails_loudly_on_cpu_tensors():
    m = RAFT(ns(small=False, mixed_precision=False)).eval()
    x = torch.zeros(1, 3, 64, 64)
    with pytest.raises(RuntimeError, match="ROCm GPU only"):
        m(x, x, iters=1, test_mode=True)


def test_training_mode_is_rejected():
    m = RAFT(ns(small=False, mixed_precision=False))
    with pytest.raises(NotImplementedError):
        m(torch.zeros(1, 3, 64, 64), torch.zeros(1, 3, 64, 64), iters=1)


def test_compat_shims_import_like_reference_demo():
    code = ("import sys; sys.path.append('core'); from raft import RAFT; from utils.utils import InputPadder; "
            "from corr import CorrBlock, AlternateCorrBlock; import raft_optical_flow_amd as r; "
            "assert RAFT is r.RAFT; sys.path.append('.'); import alt_cuda_corr; "
            "assert hasattr(alt_cuda_corr, 'forward') and hasattr(alt_cuda_corr, 'backward'); print('ok')")
    out = subprocess.run([sys.executable, "-c", code], cwd=os.path.join(REPO, "compat"), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"


def test_packing_is_deterministic_and_permutes_gru_columns():
    """The GRU split (per-iteration columns + once-per-pair inp context) covers every
    reference input column exactly once."""
    from raft_optical_flow_amd.engine import PackedUpdate
    m = RAFT(ns(small=False, mixed_precision=False))
    m.load_state_dict(seeded_state_dict(m, 0))
    pu = PackedUpdate(m.update_block, False, "cpu")
    zr, q, ctx = pu.gru[0]
    assert zr.cin_real == 256 and q.cin_real == 256 and ctx.cin_real == 128
    assert zr.n == 256 and q.n == 128 and ctx.n == 384
    g = m.update_block.gru
    w_ref = torch.cat([g.convz1.weight, g.convr1.weight], 0)   # [256, 384, 1, 5], cols h|inp|mot|flow
    # column 0 of the packed zr = h channel 0 at tap (0,0); ctx column 0 = inp channel 0
    wz = zr.weight.view(zr.weight.shape[0], 5, -1)
    assert torch.equal(wz[:256, 0, 0], w_ref[:, 0, 0, 0])
    assert torch.equal(wz[:256, 0, 128], w_ref[:, 256, 0, 0])   # first motion channel
    wc = ctx.weight.view(ctx.weight.shape[0], 5, -1)
    assert torch.equal(wc[:256, 2, 5], w_ref[:, 128 + 5, 0, 2])


def test_flo_roundtrip_and_reference_layout(tmp_path):
    """Middlebury .flo: magic, width, height, u/v interleaved (core/utils/frame_utils.py:70-99)."""
    from raft_optical_flow_amd import io as rio
    rng = np.random.default_rng(0)
    uv = rng.standard_normal((7, 11, 2)).astype(np.float32)
    p = tmp_path / "a.flo"
    rio.writeFlow(str(p), uv)
    raw = p.read_bytes()
    assert np.frombuffer(raw[:4], np.float32)[0] == np.float32(202021.25)
    assert tuple(np.frombuffer(raw[4:12], np.int32)) == (11, 7)
    assert np.array_equal(np.frombuffer(raw[12:], np.float32).reshape(7, 11, 2), uv)
    assert np.array_equal(rio.readFlow(str(p)), uv)
    rio.writeFlow(str(p), uv[..., 0], uv[..., 1])
    assert np.array_equal(rio.readFlow(str(p)), uv)
    (tmp_path / "bad.flo").write_bytes(b"\0" * 16)
    assert rio.readFlow(str(tmp_path / "bad.flo")) is None


def test_pfm_reader(tmp_path):
    from raft_optical_flow_amd import io as rio
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    p = tmp_path / "a.pfm"
    p.write_bytes(b"Pf\n4 3\n-1.0\n" + np.flipud(img).astype("<f4").tobytes())
    assert np.array_equal(rio.readPFM(str(p)), img)


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N spawns N ranks itself (one per GPU); with fewer GPUs visible it fails loudly
    before starting any, and a launcher's WORLD_SIZE that disagrees with --gpus is an error."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    env.pop("RAFT_BENCH_REHEARSE_1GPU", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 3 but only" in r.stderr
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 3" in r.stderr


class _FakePlan:
    def __init__(self):
        self.released = False

    def release(self):
        self.released = True


def test_dataparallel_replicas_keep_per_device_caches():
    """nn.DataParallel re-replicates the model on every forward (reference train.py:172,
    evaluate.py:179) by shallow-copying __dict__: each replica must reach its SOURCE's cache of its
    own device (packed weights and plans survive across forwards), have its own range-guard queue,
    and never clear or evict another device's plans."""
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False)).eval()
    r0 = m._replicate_for_data_parallel()
    r1 = m._replicate_for_data_parallel()
    r1b = r1._replicate_for_data_parallel()  # a replica of a replica still points at the source
    assert r0._source() is m and r1._source() is m and r1b._source() is m
    assert r0._pending is not m._pending and r1._pending is not r0._pending
    c0, c1 = r0._dev_cache("cuda:0"), r1._dev_cache("cuda:1")
    assert c0 is not c1
    assert c0 is m._dev_cache("cuda:0") and c1 is m._dev_cache("cuda:1") and r1b._dev_cache("cuda:1") is c1
    p0, p1 = _FakePlan(), _FakePlan()
    c0["plans"]["k"] = p0
    c1["plans"]["k"] = p1
    # new weights seen on device 1 clear only device 1's entries
    r1._release(c1["plans"])
    assert p1.released and not p0.released and "k" in c0["plans"]
    m.release_plans()
    assert p0.released and not c0["plans"]
