"""GPU parity of the sampling stage: Halton<dim> draws, scaled Panda
configurations fused with fkcc, and the valid-vertex compaction."""
import numpy as np
import pytest

from test_gpu_parity import gpu_env_from_oracle

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    assert vamp_amd.context(0) is not None
    return vamp_amd


@pytest.mark.parametrize("dim", [7, 8, 16])
@pytest.mark.parametrize("first", [1, 999_990, 1_999_995, 3_000_000])
def test_halton_bit_exact(vamp, oracle, dim, first):
    """across the 1e6-draw resets and base rotations (halton.hh:76-82)"""
    n = 4096
    got = vamp.halton(dim, first, n)
    want = oracle.halton(dim, np.arange(first, first + n))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_halton_matches_reference_pins(vamp):
    from conftest import golden
    p = golden("ref_pins.npz")
    for dim in (7, 8):
        k = p[f"halton{dim}_k"]
        got = np.concatenate([vamp.halton(dim, int(a), 1) for a in k])
        assert np.array_equal(got.view(np.uint32), p[f"halton{dim}"].view(np.uint32))


def test_sample_fkcc_matches_oracle(vamp, oracle):
    n, first = 20000, 999_000  # spans the first reset
    env_o = oracle.sphere_cage_env()
    q, ok = vamp.panda_0_0.sample_fkcc(first, n, gpu_env_from_oracle(vamp, env_o))
    qo = oracle.scale(oracle.halton(7, np.arange(first, first + n)))
    assert np.array_equal(q.view(np.uint32), qo.view(np.uint32))
    assert np.array_equal(ok, oracle.fkcc_threads(env_o, qo))


def test_compaction(vamp):
    import torch
    dev = torch.device("cuda", 0)
    n, dim = 100_003, 7
    rows = torch.rand((n, dim), device=dev)
    flags = (torch.rand(n, device=dev) < 0.37).to(torch.uint8)
    out = torch.empty_like(rows)
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    cnt = vamp.compact_device(rows.data_ptr(), flags.data_ptr(), n, dim, out.data_ptr(), idx.data_ptr())
    want = torch.nonzero(flags).flatten()
    assert cnt == want.numel()
    assert torch.equal(idx[:cnt].long(), want)
    assert torch.equal(out[:cnt], rows[want])
