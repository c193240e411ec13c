"""fedagg_reduce_rows_f32 (borrowed fp32 rows, a device table of row
pointers) through the wide per-row tiles of k_reduce_rows_ref<RefF32>
(round 5): bitwise the narrow kernel's sums (its column mapping forced with
FEDAGG_MAP, which keeps the narrow kernels), and the reference's per-column
arithmetic (acc = fl32(acc + fl32(x * fl32(w))) from +0, in arrival order,
then fl32 division by fl32(W); fedsim/utils/aggregators.py:23-40, 118-122)
restated in numpy float32 on sampled columns.

Sizes cover the 4 x 8 tile (P >= 4,188,160), the 8 x 4 tile (>= 2,094,080)
and the narrow kernels below, each with a row count that leaves a tail of
the U-row batches.
"""
import numpy as np
import pytest
import torch

from fedsim_amd import _native, ops

pytestmark = pytest.mark.gpu

MAP_VW2 = 3 << 18  # FEDAGG_MAP: two columns per lane, the narrow kernels


def _rows(P, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.empty(P, device="cuda").normal_(0, 1, generator=g) for _ in range(K)]


def _numpy_sum(rows, w, cols, acc=None, W=None):
    s = np.zeros(len(cols), np.float32) if acc is None else acc.copy()
    for r, wk in zip(rows, w):
        x = r[cols].cpu().numpy()
        s = np.float32(s + np.float32(x * np.float32(wk)))
    if W is not None:
        s = np.float32(s / np.float32(W))
    return s


@pytest.mark.parametrize("P,K", [(4_200_000, 13), (4_200_000, 14), (3_000_004, 11),
                                 (1_500_000, 9)], ids=["4x8", "4x8_tail", "8x4", "narrow"])
@pytest.mark.parametrize("finalize", [False, True], ids=["sum", "avg"])
def test_tile_rows_match_narrow_and_reference(P, K, finalize):
    rows = _rows(P, K, seed=P % 97 + K)
    wl = [float(50 + (k * 37) % 551) for k in range(K)]
    wl[3] = 0.37
    w32 = torch.tensor([ops.fl32(x) for x in wl], dtype=torch.float32, device="cuda")
    W = sum(wl) if finalize else None
    tile = torch.empty(P, device="cuda")
    narrow = torch.empty(P, device="cuda")
    ops.reduce_rows(rows, w32, tile, W=W)
    ops.reduce_rows(rows, w32, narrow, W=W, flags=MAP_VW2)
    assert torch.equal(tile.view(torch.int32), narrow.view(torch.int32))
    cols = torch.randint(0, P, (2048,), generator=torch.Generator().manual_seed(1)).cuda()
    cols = torch.cat([cols, torch.arange(P - 64, P, device="cuda")])
    want = _numpy_sum(rows, wl, cols, W=W)
    assert np.array_equal(tile[cols].cpu().numpy().view(np.int32), want.view(np.int32))


@pytest.mark.parametrize("P", [4_200_000, 3_000_004], ids=["4x8", "8x4"])
def test_tile_rows_chain_from_acc_in(P):
    """A running sum continued with acc_in (the aggregator's drains) equals one
    call over all rows; finalize on the last call."""
    K = 17
    rows = _rows(P, K, seed=5)
    wl = [float(1 + k) for k in range(K)]
    w32 = torch.tensor(wl, dtype=torch.float32, device="cuda")
    whole = torch.empty(P, device="cuda")
    ops.reduce_rows(rows, w32, whole, W=sum(wl))
    acc = torch.empty(P, device="cuda")
    ops.reduce_rows(rows[:6], w32[:6], acc)
    out = torch.empty(P, device="cuda")
    ops.reduce_rows(rows[6:], w32[6:], out, acc_in=acc, W=sum(wl))
    assert torch.equal(out.view(torch.int32), whole.view(torch.int32))


def test_tile_rows_no_rows_is_the_running_sum():
    """B = 0 with acc_in (the narrow kernels take it; the tiles need a row):
    the running sum, divided when finalize."""
    P = 4_200_000
    acc = _rows(P, 1, seed=9)[0]
    out = torch.empty(P, device="cuda")
    w32 = torch.empty(0, dtype=torch.float32, device="cuda")
    rc = _native.load().fedagg_reduce_rows_f32(
        ops.row_table([acc], acc.device).data_ptr(), w32.data_ptr(), 0, P, acc.data_ptr(),
        out.data_ptr(), ops.fl32(3.0), _native.FEDAGG_FINALIZE, ops._stream_ptr(acc.device))
    assert rc == 0
    want = acc.cpu().numpy() / np.float32(3.0)  # IEEE division per element
    assert np.array_equal(out.cpu().numpy().view(np.int32), want.view(np.int32))


@pytest.mark.parametrize("P", [4_200_000, 3_000_004], ids=["4x8", "8x4"])
def test_tile_rows_in_place_running_sum(P):
    """The aggregator's drains continue the running sum in place (out is
    acc_in, _DeviceEntry._flush_borrowed): the same bits as one call."""
    K = 19
    rows = _rows(P, K, seed=11)
    wl = [float(3 + 5 * k) for k in range(K)]
    w32 = torch.tensor(wl, dtype=torch.float32, device="cuda")
    whole = torch.empty(P, device="cuda")
    ops.reduce_rows(rows, w32, whole, W=sum(wl))
    acc = torch.empty(P, device="cuda")
    ops.reduce_rows(rows[:5], w32[:5], acc)
    ops.reduce_rows(rows[5:12], w32[5:12], acc, acc_in=acc)
    ops.reduce_rows(rows[12:], w32[12:], acc, acc_in=acc, W=sum(wl))
    assert torch.equal(acc.view(torch.int32), whole.view(torch.int32))
