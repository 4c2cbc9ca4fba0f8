"""Row moves of the device replay buffers (mfrl_amd.algo.tools) on the HIP kernel k_rows_copy
(csrc/replay_kernels.hip): every push / tight / sample of MemoryGroup and EpisodesBuffer (algo/tools.py:26-362)
is one launch that gathers whole rows of all its columns.  CUDA tensors only; a missing engine library raises.
"""
import ctypes

import torch

from . import check, lib

_MAX_COLS = 12


def rows_copy(dst, src, idx=None, src_mod=0, dst_start=0, dst_cap=0, n=None, shift_mask=0, shift=0):
    """For i < n: row (idx[i] if idx is not None else i), taken modulo src_mod if > 0, of every tensor in
    `src` -> row dst_start + i (modulo dst_cap if > 0) of the matching tensor in `dst`.  Tensors: CUDA,
    contiguous, first dimension = rows, equal row byte sizes pairwise.  Without src_mod, an index in
    [-rows, 0) counts from the end as numpy's does; any other index outside the source rows is skipped on the
    device and raised by the next check_errors() (the reference's numpy indexing raises IndexError at once;
    checking here would synchronise every move).  Columns k with bit k of shift_mask set read row idx[i] + shift
    instead (before the modulo): MemoryGroup.sample's next-state columns in the launch of the current ones."""
    assert len(dst) == len(src) and 0 < len(dst) <= _MAX_COLS
    if n is None:
        n = len(idx) if idx is not None else src[0].shape[0]
    if n == 0:
        return
    rb = []
    for d, s in zip(dst, src):
        assert d.is_cuda and s.is_cuda and d.is_contiguous() and s.is_contiguous(), "rows_copy: contiguous CUDA tensors"
        b = d.element_size() * (d[0].numel() if d.dim() > 1 else 1)
        assert b == s.element_size() * (s[0].numel() if s.dim() > 1 else 1), "rows_copy: row sizes differ"
        rb.append(b)
    if idx is not None:
        idx = idx.to(device=dst[0].device, dtype=torch.int64).contiguous()
    k = len(dst)
    src_rows = min(s.shape[0] for s in src)
    L = lib()
    L.mfx_rows_copy.restype = ctypes.c_int
    P = ctypes.c_void_p * k
    L.mfx_rows_copy_shift.restype = ctypes.c_int
    check(L.mfx_rows_copy_shift(k, P(*[d.data_ptr() for d in dst]), P(*[s.data_ptr() for s in src]),
                                (ctypes.c_int64 * k)(*rb), ctypes.c_void_p(idx.data_ptr() if idx is not None else 0),
                                ctypes.c_int64(int(src_mod)), ctypes.c_int64(int(src_rows)),
                                ctypes.c_int64(int(dst_start)), ctypes.c_int64(int(dst_cap)), ctypes.c_int64(int(n)),
                                ctypes.c_uint32(int(shift_mask)), ctypes.c_int64(int(shift)),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
          "mfx_rows_copy_shift")


def check_errors():
    """Synchronise the current stream; raise IndexError if a rows_copy since the last check met a source
    index outside its source rows (that row was skipped)."""
    L = lib()
    L.mfx_rows_copy_error.restype = ctypes.c_int
    bad = ctypes.c_int64()
    if L.mfx_rows_copy_error(ctypes.byref(bad), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) != 0:
        raise IndexError("rows_copy: source index %d out of range" % bad.value)
