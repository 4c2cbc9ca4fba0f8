"""The replay rows' HIP mover (mfx_rows_copy, csrc/replay_kernels.hip) against torch indexing: gathers with and
without an index list, modulo a source length, into a ring with wrap; column widths that take the 16-B,
4-B and byte paths (view rows of 4,732 B, int32, bool, float64 x 21).  The buffers' semantics against the
reference's own MemoryGroup / EpisodesBuffer: test_algo_gpu.py::test_device_replay_matches_reference_fixture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cols(n, gen):
    return [torch.rand((n, 13, 13, 7), generator=gen, device="cuda"),            # 4,732 B: 4-B path
            torch.randint(0, 21, (n,), generator=gen, device="cuda", dtype=torch.int32),
            torch.rand((n,), generator=gen, device="cuda") < 0.5,                 # 1 B: byte path
            torch.rand((n, 4), generator=gen, device="cuda"),                     # 16 B: 16-B path
            torch.rand((n, 21), generator=gen, device="cuda", dtype=torch.float64)]


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("n_src,n,cap,start,mod", [(1000, 1000, 0, 0, 0), (1000, 700, 2000, 1500, 0),
                                                   (300, 257, 300, 250, 300), (50, 1, 0, 7, 0), (40000, 33333, 0, 0, 0)])
def test_rows_copy_matches_torch_indexing(n_src, n, cap, start, mod, pipe, monkeypatch):
    """pipe 1: the two-rows-in-flight form (k_rows_pipe<1, 1>: one wide column, <= 64 narrow units -- these five
    columns); 0: the one-row-per-wave form (k_rows_copy, which also takes every other column shape)."""
    monkeypatch.setenv("MFX_ROWS_PIPE", pipe)
    from mfrl_amd.replay import rows_copy
    gen = torch.Generator(device="cuda").manual_seed(n + start)
    src = _cols(n_src, gen)
    n_dst = cap if cap else start + n
    dst = [torch.zeros((n_dst,) + tuple(x.shape[1:]), dtype=x.dtype, device="cuda") for x in src]
    want = [d.clone() for d in dst]
    idx = torch.randint(-3 * n_src, 3 * n_src, (n,), generator=gen, device="cuda") if mod else \
        torch.randperm(n_src, generator=gen, device="cuda")[:n]
    rows_copy(dst, src, idx, src_mod=mod, dst_start=start, dst_cap=cap)
    s = (idx % mod) if mod else idx
    d = torch.arange(n, device="cuda") + start
    if cap:
        d = d % cap
    for w, x in zip(want, src):
        w[d] = x[s]
    torch.cuda.synchronize()
    for a, b in zip(dst, want):
        assert torch.equal(a, b)
    # no index list: rows 0..n-1 in order
    dst2 = [torch.zeros_like(x[:n]) for x in src]
    rows_copy(dst2, [x[:n].contiguous() for x in src])
    torch.cuda.synchronize()
    for a, x in zip(dst2, src):
        assert torch.equal(a, x[:n])
    from mfrl_amd.replay import check_errors
    check_errors()                                      # no index was out of range


def test_rows_copy_out_of_range_index_raises():
    """An index past the source rows (numpy indexing raises IndexError in the reference's MemoryGroup) skips
    its row instead of reading out of bounds, and the next check_errors() raises with the first such index; the
    rows with valid indices are still moved and the error word is cleared by the check."""
    from mfrl_amd.replay import check_errors, rows_copy
    gen = torch.Generator(device="cuda").manual_seed(3)
    src = _cols(64, gen)
    dst = [torch.zeros((4,) + tuple(x.shape[1:]), dtype=x.dtype, device="cuda") for x in src]
    idx = torch.tensor([5, 64, 7, 1 << 40], dtype=torch.int64, device="cuda")
    rows_copy(dst, src, idx)
    with pytest.raises(IndexError, match="out of range"):
        check_errors()
    check_errors()                                      # cleared
    for a, x in zip(dst, src):
        assert torch.equal(a[0], x[5]) and torch.equal(a[2], x[7])
        assert not a[1].any() and not a[3].any()
    # numpy's negative indices count from the end (-64 is row 0, -1 row 63); -65 is out of range and is reported
    # as itself (the bad-index word once stored index + 1, so -1 read as 'none')
    for a in dst:
        a.zero_()
    rows_copy(dst, src, torch.tensor([-1, -64, -65, 3], dtype=torch.int64, device="cuda"))
    with pytest.raises(IndexError, match="index -65 out of range"):
        check_errors()
    for a, x in zip(dst, src):
        assert torch.equal(a[0], x[63]) and torch.equal(a[1], x[0]) and torch.equal(a[3], x[3])
        assert not a[2].any()
    rows_copy(dst, src, torch.tensor([2, -100], dtype=torch.int64, device="cuda"), n=2)
    with pytest.raises(IndexError, match="index -100 out of range"):
        check_errors()


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("n_src,n,mod,n_next", [(4096, 3000, 4096, 2), (300, 257, 250, 2), (1000, 5, 1000, 1),
                                                (2000, 1999, 2000, 3)])
def test_rows_copy_shifted_columns(n_src, n, mod, n_next, pipe, monkeypatch):
    """MemoryGroup.sample's fused move (mfx_rows_copy_shift): the current columns at idx and next-state copies of
    the first n_next of them at (idx + 1) % mod, in one launch.  n_next 2: two wide columns + 90 narrow units (the
    pipelined form's limits, k_rows_pipe<2, 2>); 1: k_rows_pipe<1, 1>; 3: three wide columns take k_rows_copy."""
    monkeypatch.setenv("MFX_ROWS_PIPE", pipe)
    from mfrl_amd.replay import check_errors, rows_copy
    gen = torch.Generator(device="cuda").manual_seed(n + n_next)
    src = _cols(n_src, gen)
    nxt = [src[0], src[4], src[0]][:n_next]
    cols = src + nxt
    dst = [torch.zeros((n,) + tuple(x.shape[1:]), dtype=x.dtype, device="cuda") for x in cols]
    idx = torch.randint(-2 * mod, 2 * mod, (n,), generator=gen, device="cuda")
    idx[0] = mod - 1                                    # the wrap: next row 0
    mask = ((1 << n_next) - 1) << len(src)
    rows_copy(dst, cols, idx, src_mod=mod, shift_mask=mask, shift=1)
    torch.cuda.synchronize()
    for k, (a, x) in enumerate(zip(dst, cols)):
        s = ((idx + 1) if k >= len(src) else idx) % mod
        assert torch.equal(a, x[s]), k
    check_errors()
    # without a modulo a shifted row past the source is skipped and reported as idx + shift
    for a in dst:
        a.zero_()
    rows_copy(dst, cols, torch.tensor([3, n_src - 1], dtype=torch.int64, device="cuda"), shift_mask=mask, shift=1)
    with pytest.raises(IndexError, match="index %d out of range" % n_src):
        check_errors()
    for k, (a, x) in enumerate(zip(dst, cols)):
        assert torch.equal(a[0], x[4 if k >= len(src) else 3]) and not a[1].any()
