"""Per-rank reduction stand-in for bench.py's CPU/gloo launcher rehearsal
(``--rehearsal-stub bench_stub:reduce``).  Test infrastructure: it lets the
launcher, the rank environment, the collectives and the one-line contract run
without a GPU; no number it produces is a measurement."""
import torch


def reduce(X, w32, out, acc_in, W):
    s = (X * w32[: X.shape[0], None]).sum(0)
    if acc_in is not None:
        s = s + acc_in
    if W is not None:
        s = s / float(W)
    out.copy_(s)
    return out


def fail_on_rank1(X, w32, out, acc_in, W):
    """A rank that dies mid-run: the launcher must end the others and fail."""
    import os

    if os.environ.get("RANK") == "1":
        raise RuntimeError("injected failure on rank 1")
    return reduce(X, w32, out, acc_in, W)
