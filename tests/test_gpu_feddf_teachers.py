"""FedDF's teacher ensemble on the matrix cores (fedagg_teacher_linear_f32,
fedagg_teacher_conv2d_f32, fedagg_pad_lrn_maxpool_f32,
training/teacher_program.py): the layer kernels against an fp64 reference
within the f32 dot-product error bound and bit for bit against the C
oracle's fmaf chains, over ragged shapes; the pad / LRN / max-pool pass
against the C oracle and torch's own ops; the traced replay of whole models
(MLP, CNNs incl. the reference's SimpleCNN2) over K stacked teachers against
each teacher's own forward; and the ensemble keeping the kernel path after
its first-batch check.  Reference: fedsim/distributed/centralized/training/
feddf.py:117-122, fedsim/models/simple_models.py:165-255."""
import numpy as np
import pytest
import torch
from torch.func import functional_call

from test_teacher_program import Cnn, Cnn2, Mlp, Tiny

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("M,in_f,out_f", [(1, 1, 1), (63, 3, 65), (64, 37, 11), (65, 784, 200),
                                          (130, 200, 10), (7, 2304, 384), (64, 33, 129)])
@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("bias,relu", [(True, False), (False, True), (True, True)])
def test_teacher_linear_kernel(M, in_f, out_f, shared, bias, relu):
    from fedsim_amd import ops

    g = torch.Generator(device=DEV).manual_seed(M * 131 + in_f * 7 + out_f)
    K = 5
    pad = 3  # the layer's parameters start at an odd offset of the teacher's vector
    P = pad + in_f * out_f + (out_f if bias else 0) + 2
    slab = torch.randn(K, P, device=DEV, generator=g)
    x = torch.randn((M, in_f) if shared else (K, M, in_f), device=DEV, generator=g)
    b_off = pad + in_f * out_f if bias else -1
    y = ops.teacher_linear(x, slab, pad, b_off, in_f, out_f, shared=shared, relu=relu)
    W = slab[:, pad:pad + in_f * out_f].view(K, out_f, in_f).double()
    xs = (x.expand(K, M, in_f) if shared else x).double()
    y64 = torch.einsum("kmi,koi->kmo", xs, W)
    absum = torch.einsum("kmi,koi->kmo", xs.abs(), W.abs())
    if bias:
        bb = slab[:, b_off:b_off + out_f].double().view(K, 1, out_f)
        y64 = y64 + bb
        absum = absum + bb.abs()
    if relu:
        y64 = y64.clamp_min(0)
    gamma = (in_f + 1) * 2.0 ** -24 / (1 - (in_f + 1) * 2.0 ** -24)
    err = (y.double() - y64).abs()
    assert bool((err <= gamma * absum + 1e-30).all()), float((err - gamma * absum).max())


@pytest.mark.parametrize("cls,shape", [(Tiny, (64, 37)), (Mlp, (100, 1, 8, 8)),
                                       (Cnn, (64, 3, 8, 8)), (Cnn2, (64, 3, 8, 8))])
def test_program_replays_each_teachers_forward(cls, shape):
    from fedsim_amd.distributed.centralized.training import teacher_program as TP
    from fedsim_amd.utils import vector_to_named_parameters_like

    torch.manual_seed(1)
    model = cls().to(DEV)
    named = list(model.named_parameters())
    K = 70
    base = torch.cat([p.detach().reshape(-1) for _, p in named])
    slab = torch.stack([base + 0.05 * torch.randn_like(base) for _ in range(K)])
    prog = TP.build(model, named, slab)
    assert prog is not None
    x = torch.randn(*shape, device=DEV)
    got = prog(x)
    want = torch.stack([functional_call(model, vector_to_named_parameters_like(slab[k], named),
                                        (x,)) for k in range(K)])
    rel = float(torch.linalg.vector_norm((got - want).double()) /
                torch.linalg.vector_norm(want.double()))
    assert rel <= 1e-5, rel
    assert prog.linear_launches == sum(isinstance(m, torch.nn.Linear) for m in model.modules())
    assert prog.conv_launches == sum(isinstance(m, torch.nn.Conv2d) for m in model.modules())
    assert prog.pool_launches == {Tiny: 0, Mlp: 0, Cnn: 2, Cnn2: 2}[cls]


def test_ensemble_keeps_the_matrix_core_path():
    """The ensemble's first batch checks the replay against the vmap'd
    forward and keeps it; the mean is the exact weight-1 mean of the replay's
    logits (fedagg_reduce_f32), bitwise vs the oracle."""
    from conftest import bits
    from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble
    from oracle import ref

    torch.manual_seed(2)
    model = Cnn().to(DEV)
    base = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    teachers = [base + 0.05 * torch.randn_like(base) for _ in range(33)]
    ens = TeacherEnsemble(model, teachers, DEV)
    assert ens.program is not None
    x = torch.randn(64, 3, 8, 8, device=DEV)
    for _ in range(2):
        mean = ens.mean_logits(x)
        assert ens.program is not None and ens._checked
    logits = ens.program(x).reshape(33, -1).cpu().numpy()
    exp = ref.reduce(logits, [1] * 33, W=33)
    np.testing.assert_array_equal(bits(mean.reshape(-1).cpu().numpy()), bits(exp))


@pytest.mark.parametrize("M,in_f,out_f", [(1, 1, 1), (63, 3, 65), (64, 37, 11), (65, 784, 200),
                                          (130, 200, 10), (7, 33, 129)])
@pytest.mark.parametrize("shared", [True, False])
def test_teacher_linear_kernel_is_the_fmaf_chain(M, in_f, out_f, shared):
    """Bitwise against the C oracle's restatement (oracle/fedagg_ref.c
    ref_teacher_linear_f32): each output is an f32 fmaf chain over the inputs
    in order, then one bias add -- what v_mfma_f32_16x16x4_f32 computes."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    g = torch.Generator(device=DEV).manual_seed(M + 17 * in_f + out_f)
    K = 3
    P = 5 + in_f * out_f + out_f
    slab = torch.randn(K, P, device=DEV, generator=g)
    x = torch.randn((M, in_f) if shared else (K, M, in_f), device=DEV, generator=g)
    for relu in (False, True):
        y = ops.teacher_linear(x, slab, 5, 5 + in_f * out_f, in_f, out_f, shared=shared,
                               relu=relu)
        exp = ref.teacher_linear(x.cpu().numpy(), slab.cpu().numpy(), 5, 5 + in_f * out_f, in_f,
                                 out_f, shared, relu)
        np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(exp))


@pytest.mark.parametrize("w_off,P_pad", [(0, 0), (4, 0), (8, 2), (0, 1)])
def test_teacher_linear_aligned_rows_bitwise(w_off, P_pad):
    """16-byte staging loads (rows of x and of the teacher's W 16-B aligned;
    with P % 4 = 2 every other teacher takes the 4-byte loads): bitwise vs
    the C oracle's fmaf chain at SimpleMLP's and SimpleCNN's layer sizes."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    for M, in_f, out_f in ((64, 784, 200), (64, 3136, 80), (70, 32, 130)):
        g = torch.Generator(device=DEV).manual_seed(in_f + out_f + w_off + P_pad)
        K = 4
        P = (w_off + in_f * out_f + out_f + 3) // 4 * 4 + P_pad
        slab = torch.randn(K, P, device=DEV, generator=g)
        for shared in (True, False):
            x = torch.randn((M, in_f) if shared else (K, M, in_f), device=DEV, generator=g)
            y = ops.teacher_linear(x, slab, w_off, w_off + in_f * out_f, in_f, out_f,
                                   shared=shared, relu=True)
            exp = ref.teacher_linear(x.cpu().numpy(), slab.cpu().numpy(), w_off,
                                     w_off + in_f * out_f, in_f, out_f, shared, True)
            np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(exp))


def test_padded_row_pitch_slab_same_bits():
    """TeacherEnsemble pads each teacher's row to 16 bytes; the Linear and
    Conv2d kernels read a row-strided [K, P] view (row pitch passed as the
    teachers' stride) with the same results as a contiguous slab."""
    from conftest import bits
    from fedsim_amd import ops
    from fedsim_amd.distributed.centralized.training.feddf import _stack_rows

    g = torch.Generator(device=DEV).manual_seed(11)
    K, P = 5, 199_210  # SimpleMLP's P: odd rows misaligned in a contiguous slab
    rows = [torch.randn(P, device=DEV, generator=g) for _ in range(K)]
    padded = _stack_rows(rows, DEV)
    assert padded.stride(0) % 4 == 0 and padded.stride(0) >= P
    dense = torch.stack(rows)
    x = torch.randn(64, 784, device=DEV, generator=g)
    a = ops.teacher_linear(x, padded, 0, 784 * 200, 784, 200, shared=True, relu=True)
    b = ops.teacher_linear(x, dense, 0, 784 * 200, 784, 200, shared=True, relu=True)
    np.testing.assert_array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))
    xc = torch.randn(8, 3, 24, 24, device=DEV, generator=g)
    a = ops.teacher_conv2d(xc, padded, 1, 4801, 64, (5, 5), (1, 1), (2, 2, 2, 2), shared=True)
    b = ops.teacher_conv2d(xc, dense, 1, 4801, 64, (5, 5), (1, 1), (2, 2, 2, 2), shared=True)
    np.testing.assert_array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))


def test_teacher_linear_random_shapes_bitwise():
    """Random layer shapes, offsets and teacher counts (seeded), bitwise vs
    the C oracle's fmaf chain, including special values in the inputs."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    rng = np.random.default_rng(2026)
    for _ in range(40):
        K = int(rng.integers(1, 6))
        M = int(rng.integers(1, 150))
        in_f = int(rng.integers(1, 300))
        out_f = int(rng.integers(1, 150))
        w_off = int(rng.integers(0, 9))
        bias = bool(rng.integers(0, 2))
        P = w_off + in_f * out_f + (out_f if bias else 0) + int(rng.integers(0, 5))
        slab = rng.standard_normal((K, P)).astype(np.float32)
        shared = bool(rng.integers(0, 2))
        x = rng.standard_normal((M, in_f) if shared else (K, M, in_f)).astype(np.float32)
        x.reshape(-1)[:: max(1, x.size // 7)] = np.float32(-0.0)
        relu = bool(rng.integers(0, 2))
        b_off = w_off + in_f * out_f if bias else -1
        y = ops.teacher_linear(torch.from_numpy(x).to(DEV), torch.from_numpy(slab).to(DEV),
                               w_off, b_off, in_f, out_f, shared=shared, relu=relu)
        exp = ref.teacher_linear(x, slab, w_off, b_off, in_f, out_f, shared, relu)
        np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(exp),
                                      err_msg=f"K={K} M={M} in={in_f} out={out_f}")


# (M, C, H, W, OC, kernel, stride, pads=(top, bottom, left, right))
CONV_CASES = [
    (2, 3, 24, 24, 64, (5, 5), (1, 1), (2, 2, 2, 2)),    # SimpleCNN2 conv1 (R = 75: 16-stages)
    (2, 64, 12, 12, 64, (5, 5), (1, 1), (2, 2, 2, 2)),   # SimpleCNN2 conv2 (R = 1600)
    (3, 1, 28, 28, 32, (5, 5), (1, 1), (2, 2, 2, 2)),    # SimpleCNN conv1 on MNIST
    (1, 5, 7, 9, 5, (3, 4), (1, 1), (1, 1, 1, 2)),       # padding="same", even kernel width
    (4, 7, 11, 10, 100, (3, 3), (2, 2), (1, 1, 1, 1)),   # stride 2, two channel tiles
    (5, 2, 6, 6, 3, (1, 1), (1, 1), (0, 0, 0, 0)),       # 1x1
    (1, 33, 5, 5, 65, (5, 5), (1, 3), (0, 0, 4, 0)),     # R = 825, ragged everything
    # the LDS-resident kernel (stride 1, 3x3 / 5x5): chunk tails, image slots
    (9, 5, 12, 12, 64, (5, 5), (1, 1), (2, 2, 2, 2)),    # C = 5: a one-channel last chunk
    (3, 2, 10, 7, 130, (3, 3), (1, 1), (1, 1, 1, 1)),    # chunks of 2, three channel tiles
    (40, 6, 4, 4, 17, (3, 3), (1, 1), (0, 2, 2, 0)),     # 16-pixel images: 17 per tile
    (2, 8, 9, 11, 64, (5, 5), (1, 1), (0, 4, 3, 1)),     # asymmetric padding
    (1, 4, 20, 20, 8, (5, 5), (1, 1), (0, 0, 0, 0)),     # valid conv, one image
    (2, 4, 40, 40, 8, (5, 5), (1, 1), (2, 2, 2, 2)),     # tile too big for LDS: gather kernel
    # every channel staged (C = 1 / 3): flattened (c, kh, kw) pairs, odd R tails
    (5, 3, 9, 9, 70, (3, 3), (1, 1), (1, 1, 1, 1)),      # R = 27, five image slots, 2 oc tiles
    (2, 1, 30, 30, 16, (3, 3), (1, 1), (0, 0, 0, 0)),    # R = 9, valid conv
    (3, 3, 16, 16, 64, (5, 5), (1, 1), (0, 4, 1, 3)),    # asymmetric padding
    (1, 3, 30, 30, 33, (5, 5), (1, 1), (2, 2, 2, 2)),    # one image, 16 staging registers
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("shared", [True, False])
def test_teacher_conv2d_kernel_is_the_fmaf_chain(case, shared):
    """Bitwise against the C oracle's restatement (oracle/fedagg_ref.c
    ref_teacher_conv2d_f32): each output is the fmaf chain over (c, kh, kw)
    in order (zeros outside the input), then one bias add, then ReLU -- the
    implicit GEMM on v_mfma_f32_32x32x2_f32; and within the f32 dot-product
    bound of an fp64 convolution."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    M, C, H, W, OC, kern, stride, pads = case
    g = torch.Generator(device=DEV).manual_seed(M * 7 + C * 13 + OC)
    K = 3
    R = C * kern[0] * kern[1]
    w_off = 5
    P = w_off + OC * R + OC + 3
    slab = torch.randn(K, P, device=DEV, generator=g)
    x = torch.randn((M, C, H, W) if shared else (K, M, C, H, W), device=DEV, generator=g)
    x.view(-1)[:: 97] = -0.0
    for gather in (False, True):
        cc = ops.conv_order(x.shape, OC, kern, stride, pads, gather=gather)
        for bias, relu in ((True, False), (False, True), (True, True)):
            b_off = w_off + OC * R if bias else -1
            y = ops.teacher_conv2d(x, slab, w_off, b_off, OC, kern, stride, pads, shared=shared,
                                   relu=relu, gather=gather)
            exp = ref.teacher_conv2d(x.cpu().numpy(), slab.cpu().numpy(), w_off, b_off, OC,
                                     kern, stride, pads, shared, relu, cc=cc)
            assert y.shape == exp.shape
            np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(exp),
                                          err_msg=f"gather={gather} cc={cc}")
    # and the chain is a convolution: fp64 within gamma_R
    F = torch.nn.functional
    Wt = slab[:, w_off:w_off + OC * R].view(K, OC, C, *kern).double()
    bt = slab[:, w_off + OC * R:w_off + OC * R + OC].double()
    xs = (x.expand(K, *x.shape) if shared else x).double()
    t, b, l, r = pads
    y = ops.teacher_conv2d(x, slab, w_off, w_off + OC * R, OC, kern, stride, pads, shared=shared)
    gamma = (R + 1) * 2.0 ** -24 / (1 - (R + 1) * 2.0 ** -24)
    for k in range(K):
        xp = F.pad(xs[k], (l, r, t, b))
        y64 = F.conv2d(xp, Wt[k], bt[k], stride)
        absum = F.conv2d(xp.abs(), Wt[k].abs(), bt[k].abs(), stride)
        err = (y[k].double() - y64).abs()
        assert bool((err <= gamma * absum + 1e-30).all())


def test_teacher_conv2d_random_shapes_bitwise():
    """Random conv geometries, offsets and teacher counts (seeded), bitwise
    vs the C oracle, special values in the input included."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    rng = np.random.default_rng(355)
    lds_cases = 0
    for it in range(40):
        K = int(rng.integers(1, 4))
        M = int(rng.integers(1, 4))
        C = int(rng.integers(1, 20))
        H, W = int(rng.integers(1, 14)), int(rng.integers(1, 14))
        kh, kw = int(rng.integers(1, min(H, 5) + 1)), int(rng.integers(1, min(W, 5) + 1))
        sh, sw = int(rng.integers(1, 3)), int(rng.integers(1, 3))
        if it % 3 == 0 and min(H, W) >= 3:  # a geometry the LDS-resident kernel takes
            kh = kw = 5 if min(H, W) >= 5 and it % 2 else 3
            sh = sw = 1
        pads = tuple(int(v) for v in rng.integers(0, 3, 4))
        OC = int(rng.integers(1, 80))
        R = C * kh * kw
        w_off = int(rng.integers(0, 7))
        bias = bool(rng.integers(0, 2))
        P = w_off + OC * R + (OC if bias else 0) + int(rng.integers(0, 4))
        slab = rng.standard_normal((K, P)).astype(np.float32)
        shared = bool(rng.integers(0, 2))
        x = rng.standard_normal((M, C, H, W) if shared else (K, M, C, H, W)).astype(np.float32)
        x.reshape(-1)[:: max(1, x.size // 5)] = np.float32(-0.0)
        relu = bool(rng.integers(0, 2))
        b_off = w_off + OC * R if bias else -1
        cc = ops.conv_order(x.shape, OC, (kh, kw), (sh, sw), pads)
        lds_cases += cc > 0
        y = ops.teacher_conv2d(torch.from_numpy(x).to(DEV), torch.from_numpy(slab).to(DEV),
                               w_off, b_off, OC, (kh, kw), (sh, sw), pads, shared=shared,
                               relu=relu)
        exp = ref.teacher_conv2d(x, slab, w_off, b_off, OC, (kh, kw), (sh, sw), pads, shared,
                                 relu, cc=cc)
        np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(exp),
                                      err_msg=f"K={K} M={M} C={C} HxW={H}x{W} k={kh}x{kw} "
                                              f"s={sh}x{sw} pads={pads} OC={OC} cc={cc}")
    assert lds_cases >= 5  # the LDS-resident kernel is among them


@pytest.mark.parametrize("M,C,H,W,OC,pads,K", [
    (64, 3, 24, 24, 64, (2, 2, 2, 2), 30),    # SimpleCNN2 conv1
    (64, 1, 28, 28, 32, (1, 1, 1, 1), 50),    # SimpleCNN conv1: OC = 32, upper half skipped
    (33, 3, 17, 13, 70, (2, 2, 2, 2), 200),   # ragged last tiles, two channel tiles
    (9, 3, 20, 20, 20, (2, 2, 2, 2), 40),     # OC <= 32: 128 pixels per wave, ragged
])
def test_flat_conv_matches_the_gather_chain(M, C, H, W, OC, pads, K):
    """The 1- / 3-channel LDS conv (every channel staged, k pairs over the
    flattened (c, kh, kw) index) and the im2col-gather kernel run the same
    chain: bit for bit over every teacher at the reference's layer sizes;
    the first and last teacher also against the C oracle."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    g = torch.Generator(device=DEV).manual_seed(M + C + OC + K)
    kern = (5, 5)
    R = C * 25
    P = 3 + OC * R + OC
    slab = torch.randn(K, P, device=DEV, generator=g)
    x = torch.randn(M, C, H, W, device=DEV, generator=g)
    assert ops.conv_order(x.shape, OC, kern, (1, 1), pads) == 0
    y = ops.teacher_conv2d(x, slab, 3, 3 + OC * R, OC, kern, (1, 1), pads, shared=True, relu=True)
    yg = ops.teacher_conv2d(x, slab, 3, 3 + OC * R, OC, kern, (1, 1), pads, shared=True,
                            relu=True, gather=True)
    assert torch.equal(y.view(torch.int32), yg.view(torch.int32))
    ends = slab[[0, K - 1]].cpu().numpy()
    exp = ref.teacher_conv2d(x.cpu().numpy(), ends, 3, 3 + OC * R, OC, kern, (1, 1), pads, True,
                             True, cc=0)
    np.testing.assert_array_equal(bits(y[[0, K - 1]].cpu().numpy()), bits(exp))


# (shape, pads, lrn, pool)
POOL_CASES = [
    ((4, 64, 24, 24), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0)),  # SimpleCNN2 1
    ((4, 64, 12, 12), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0)),  # SimpleCNN2 2
    ((3, 32, 28, 28), (0, 0, 0, 0), None, (2, 2, 2, 2, 1, 1)),                       # SimpleCNN
    ((2, 5, 7, 9), (1, 2, 0, 3), (3, 0.01, 0.5, 2.0), None),                         # no pool
    ((2, 3, 6, 5), (0, 0, 0, 0), (5, 1.0, 1.25, 0.5), (2, 3, 1, 2, 1, 1)),           # C < size
    ((1, 70, 30, 31), (2, 0, 1, 1), (4, 1e-4, 0.75, 1.0), (3, 2, 3, 2, 1, 0)),       # ragged blocks
    ((2, 20, 9, 9), (1, 1, 1, 1), (7, 2e-3, 0.6, 1.5), (3, 3, 3, 3, 1, 1)),          # any-size LRN
    ((1, 3, 120, 120), (0, 0, 0, 0), (3, 1e-3, 0.75, 1.0), (2, 2, 2, 2, 0, 0)),      # 1 channel / WG
]


@pytest.mark.parametrize("case", POOL_CASES)
def test_pad_lrn_maxpool_kernel(case):
    """Against the C oracle (pooling, padding and the channel window exactly;
    the LRN's powf within 2 ulps of the host's) and against torch's own
    F.pad -> F.local_response_norm -> F.max_pool2d on the same GPU."""
    from fedsim_amd import ops
    from oracle import ref

    shape, pads, lrn, pool = case
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    x = torch.randn(*shape, device=DEV, generator=g) * 3
    x.view(-1)[:: 89] = 0.0
    y = ops.pad_lrn_maxpool(x, pads, lrn, pool)
    exp = ref.pad_lrn_maxpool(x.cpu().numpy(), pads, lrn, pool)
    assert y.shape == exp.shape
    got = y.cpu().numpy()
    if lrn is None:
        np.testing.assert_array_equal(got, exp)
    else:
        ulp = np.spacing(np.abs(exp).astype(np.float32))
        assert float((np.abs(got - exp) / ulp).max()) <= 8.0  # hardware exp2 / log2 power
    F = torch.nn.functional
    t, b, l, r = pads
    want = F.pad(x, (l, r, t, b))
    if lrn is not None:
        want = F.local_response_norm(want, lrn[0], alpha=lrn[1], beta=lrn[2], k=lrn[3])
    if pool is not None:
        kh, kw, sh, sw, ph, pw = pool
        want = F.max_pool2d(want, (kh, kw), (sh, sw), (ph, pw))
    torch.testing.assert_close(y, want, rtol=1e-6, atol=0)
    # the sliding channel window and the per-block kernels: the same bits
    from conftest import bits

    y_planes = ops.pad_lrn_maxpool(x, pads, lrn, pool, planes=True)
    np.testing.assert_array_equal(bits(got), bits(y_planes.cpu().numpy()))


# sliding-window pass: every plane size class (1..4 x 256 positions), LRN
# sizes 0 / 3 / 4 / 5, ragged last blocks, channel groups at few images
# (group boundaries inside the LRN window), C below the block
SLIDE_CASES = [
    ((1, 64, 24, 24), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0)),
    ((7, 37, 12, 12), (0, 1, 0, 1), (4, 0.001 / 9, 0.75, 1.0), (3, 3, 2, 2, 0, 0)),
    ((3, 19, 20, 20), (1, 1, 1, 1), (3, 0.01, 0.5, 2.0), (2, 2, 2, 2, 0, 0)),
    ((2, 45, 27, 27), (0, 1, 2, 0), (5, 1e-3, 0.75, 1.0), (3, 3, 2, 2, 1, 1)),
    ((5, 11, 31, 32), (0, 0, 0, 1), (4, 2e-3, 0.6, 1.5), (2, 3, 2, 1, 1, 0)),
    ((600, 9, 10, 10), (0, 0, 0, 0), None, (2, 2, 2, 2, 0, 0)),
    ((2, 2, 16, 16), (1, 0, 0, 1), (5, 1.0, 1.25, 0.5), None),
]


@pytest.mark.parametrize("case", SLIDE_CASES)
def test_pad_lrn_maxpool_slide_vs_planes(case):
    """The sliding channel window (default for planes <= 1024 positions)
    against the per-block kernels, bit for bit, and against the C oracle."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    shape, pads, lrn, pool = case
    g = torch.Generator(device=DEV).manual_seed(7 * sum(shape))
    x = torch.randn(*shape, device=DEV, generator=g) * 2
    x.view(-1)[:: 53] = 0.0
    y = ops.pad_lrn_maxpool(x, pads, lrn, pool)
    y_planes = ops.pad_lrn_maxpool(x, pads, lrn, pool, planes=True)
    np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(y_planes.cpu().numpy()))
    exp = ref.pad_lrn_maxpool(x.cpu().numpy(), pads, lrn, pool)
    got = y.cpu().numpy()
    if lrn is None:
        np.testing.assert_array_equal(got, exp)
    else:
        ulp = np.spacing(np.abs(exp).astype(np.float32))
        assert float((np.abs(got - exp) / ulp).max()) <= 8.0


P3 = ((0, 1, 0, 1), (3, 3, 2, 2, 0, 0))   # SimpleCNN2's pad + 3 x 3 / 2 pool
P2 = ((0, 0, 0, 0), (2, 2, 2, 2, 1, 1))   # SimpleCNN's 2 x 2 / 2 pool, padding 1


@pytest.mark.parametrize("shape,lrn,geom", [
    ((3, 64, 24, 24), None, P3),                          # SimpleCNN2 pool1 geometry, no LRN
    ((3, 64, 24, 24), (4, 0.001 / 9, 0.75, 1.0), P3),     # pool1 as the model runs it
    ((5, 64, 12, 12), (4, 0.001 / 9, 0.75, 1.0), P3),     # pool2
    ((2, 37, 12, 12), None, P3),                          # ragged last channel block
    ((4, 64, 12, 12), None, P2),                          # SimpleCNN pool2: -inf border
    ((3, 32, 26, 26), None, P2),                          # SimpleCNN pool1 shape, 4 x 256 planes
    ((2, 21, 9, 11), (3, 0.01, 0.5, 2.0), ((1, 0, 2, 1), (3, 3, 2, 2, 1, 1))),  # both paddings
])
def test_pad_lrn_maxpool_signed_zeros_and_nans(shape, lrn, geom):
    """The mapped 2 x 2 / 3 x 3 pools' maximum3 fast path falls back to the
    scan rule for windows holding a -0 or a NaN, and the pool padding is a
    -inf border: with many +-0 windows (first zero in window order decides
    the sign) and NaNs sprinkled in, the sliding pass is bit for bit the
    per-block pass (pool_planes' scan) and, without LRN, the C oracle."""
    from conftest import bits
    from fedsim_amd import ops
    from oracle import ref

    g = torch.Generator(device=DEV).manual_seed(sum(shape) + (lrn is None))
    x = torch.randn(*shape, device=DEV, generator=g)
    x = torch.where(x < 0.3, torch.zeros_like(x), x)        # most windows all zero
    sign = torch.rand(*shape, device=DEV, generator=g) < 0.5
    x = torch.where(sign & (x == 0), -x, x)                 # -0 / +0 mixed
    x.view(-1)[:: 1013] = float("nan")
    pads, pool = geom
    y = ops.pad_lrn_maxpool(x, pads, lrn, pool)
    y_planes = ops.pad_lrn_maxpool(x, pads, lrn, pool, planes=True)
    got = bits(y.cpu().numpy())
    np.testing.assert_array_equal(got, bits(y_planes.cpu().numpy()))
    assert (got == np.uint32(0x80000000)).any() and (got == 0).any()  # both zero signs out
    assert np.isnan(y.cpu().numpy()).any()
    if lrn is None:
        exp = ref.pad_lrn_maxpool(x.cpu().numpy(), pads, lrn, pool)
        np.testing.assert_array_equal(got, bits(exp))


def test_pad_lrn_maxpool_special_values():
    """NaN propagates through the max pool and +-inf through pooling without
    LRN, as torch's max_pool2d does; 5-D input (teachers x images)."""
    from fedsim_amd import ops

    x = torch.randn(2, 3, 4, 6, 6, device=DEV)
    x[0, 1, 2, 3, 3] = float("nan")
    x[1, 0, 0, 0, 0] = float("inf")
    x[1, 2, 1, 5, 5] = float("-inf")
    y = ops.pad_lrn_maxpool(x, (0, 1, 0, 1), None, (3, 3, 2, 2, 0, 0))
    want = torch.nn.functional.max_pool2d(
        torch.nn.functional.pad(x.view(6, 4, 6, 6), (0, 1, 0, 1)), 3, 2).view(2, 3, 4, 3, 3)
    torch.testing.assert_close(y, want, equal_nan=True, rtol=0, atol=0)


def test_kernel_shape_guards():
    """Rejected before any launch: a pool plane above 64 KiB of LDS, a pool
    padding above half the kernel, and conv layers outside the teacher's
    vector."""
    import ctypes

    from fedsim_amd import _native, ops

    x = torch.zeros(1, 1, 200, 200, device=DEV)
    with pytest.raises(ValueError):
        ops.pad_lrn_maxpool(x, (0, 0, 0, 0), None, (2, 2, 2, 2, 0, 0))
    with pytest.raises(ValueError):
        ops.pad_lrn_maxpool(torch.zeros(1, 1, 8, 8, device=DEV), (0, 0, 0, 0), None,
                            (2, 2, 2, 2, 2, 2))
    slab = torch.zeros(2, 10, device=DEV)
    with pytest.raises(ValueError):
        ops.teacher_conv2d(torch.zeros(1, 1, 4, 4, device=DEV), slab, 0, -1, 2, (3, 3), (1, 1),
                           (0, 0, 0, 0), shared=True)
    shape = _native.Conv2dShape(1, 1, 4, 4, 1, 3, 3, 1, 1, 0, 0, 2, 2)
    rc = _native.load().fedagg_teacher_conv2d_f32(0, 0, slab.data_ptr(), 10, 5, -1, 2,
                                                  ctypes.byref(shape), 0, 0, None)
    assert rc == _native.FEDAGG_EINVAL


def test_simplecnn2_replay_at_reference_size():
    """The reference's SimpleCNN2 (CIFAR-100 head) at its own input size over
    40 teachers: the replay with both convolutions, both pad / LRN / pool
    passes and the three Linear layers on this library's kernels matches
    each teacher's own forward normwise."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from bench_feddf_teachers import SimpleCNN2
    from fedsim_amd.distributed.centralized.training import teacher_program as TP
    from fedsim_amd.utils import vector_to_named_parameters_like

    torch.manual_seed(5)
    model = SimpleCNN2().to(DEV)
    named = list(model.named_parameters())
    K = 40
    base = torch.cat([p.detach().reshape(-1) for _, p in named])
    slab = torch.stack([base + 0.05 * torch.randn_like(base) for _ in range(K)])
    prog = TP.build(model, named, slab)
    x = torch.randn(64, 3, 24, 24, device=DEV)
    got = prog(x)
    want = torch.stack([functional_call(model, vector_to_named_parameters_like(slab[k], named),
                                        (x,)) for k in range(K)])
    rel = float(torch.linalg.vector_norm((got - want).double()) /
                torch.linalg.vector_norm(want.double()))
    assert rel <= 1e-5, rel
    assert (prog.conv_launches, prog.pool_launches, prog.linear_launches) == (2, 2, 3)


@pytest.mark.parametrize("M,C,H,W,OC,pads,K,pp,relu,shared", [
    (64, 1, 28, 28, 32, (1, 1, 1, 1), 40, 1, True, True),    # SimpleCNN conv1 -> pool(2, 2, pad 1)
    (64, 1, 28, 28, 32, (1, 1, 1, 1), 3, 1, True, False),    # per-teacher inputs
    (64, 3, 24, 24, 64, (2, 2, 2, 2), 20, 0, True, True),    # RGB, both channel halves, pad 0
    (7, 3, 17, 13, 70, (2, 2, 2, 2), 30, 1, False, True),    # odd planes, no ReLU, 2 oc tiles
    (5, 1, 9, 12, 20, (1, 1, 1, 1), 9, 0, False, False),     # OH = 7 odd: pool drops a row
    (1, 1, 6, 6, 3, (1, 1, 1, 1), 2, 1, True, True),         # one image, a few windows
])
def test_conv_with_fused_maxpool_is_conv_then_pool_bitwise(M, C, H, W, OC, pads, K, pp, relu,
                                                           shared):
    """FEDAGG_CONV_MAXPOOL2: the 2 x 2 / stride 2 max pool in the flat conv's
    store gives the same bits as the conv kernel followed by the pool pass
    (and torch's max_pool2d on that output), for both pool paddings, with
    and without the fused ReLU, and the pooled shape torch gives."""
    from fedsim_amd import ops

    g = torch.Generator(device=DEV).manual_seed(M + C + OC + K + pp)
    kern = (5, 5)
    R = C * 25
    P = 3 + OC * R + OC
    slab = torch.randn(K, P, device=DEV, generator=g)
    x = torch.randn(M, C, H, W, device=DEV, generator=g)
    if not shared:
        x = x.expand(K, *x.shape).contiguous() + 0.1 * torch.randn(K, *x.shape, device=DEV,
                                                                    generator=g)
    pool = (2, 2, 2, 2, pp, pp)
    assert ops.conv_pool_fusable(x.shape, OC, kern, (1, 1), pads, pool)
    y = ops.teacher_conv2d(x, slab, 3, 3 + OC * R, OC, kern, (1, 1), pads, shared=shared,
                           relu=relu)
    want = ops.pad_lrn_maxpool(y, (0, 0, 0, 0), None, pool)
    got = ops.teacher_conv2d(x, slab, 3, 3 + OC * R, OC, kern, (1, 1), pads, shared=shared,
                             relu=relu, pool=pool)
    assert got.shape == want.shape
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))
    tw = torch.nn.functional.max_pool2d(y.reshape(-1, *y.shape[-2:]), 2, 2, pp)
    assert torch.equal(got.reshape(tw.shape).view(torch.int32), tw.view(torch.int32))


def test_conv_with_fused_maxpool_special_values():
    """NaN / inf in a teacher's weights reach the pooled output as the
    two-pass result has them (max_pool2d's NaN rule, in window order)."""
    from fedsim_amd import ops

    g = torch.Generator(device=DEV).manual_seed(99)
    M, C, H, W, OC, K = 4, 1, 10, 10, 8, 3
    R = C * 25
    P = OC * R + OC
    slab = torch.randn(K, P, device=DEV, generator=g)
    slab[0, 0] = float("nan")                # channel 0 of teacher 0: NaN everywhere
    slab[1, R * 3 + 7] = float("inf")        # channel 3 of teacher 1: +-inf / NaN mixes
    slab[2, OC * R + 5] = float("-inf")      # bias of channel 5, teacher 2: -inf plane
    x = torch.randn(M, C, H, W, device=DEV, generator=g)
    x[1, 0, 4, 4] = 0.0
    for relu in (False, True):
        for pp in (0, 1):
            pool = (2, 2, 2, 2, pp, pp)
            y = ops.teacher_conv2d(x, slab, 0, OC * R, OC, (5, 5), (1, 1), (1, 1, 1, 1),
                                   shared=True, relu=relu)
            want = ops.pad_lrn_maxpool(y, (0, 0, 0, 0), None, pool)
            got = ops.teacher_conv2d(x, slab, 0, OC * R, OC, (5, 5), (1, 1), (1, 1, 1, 1),
                                     shared=True, relu=relu, pool=pool)
            assert torch.equal(got.view(torch.int32), want.view(torch.int32)), (relu, pp)


def test_fused_maxpool_rejected_where_not_taken():
    """Only the flat (1- / 3-channel) kernel fuses the pool; anything else is
    refused before a launch (the replay keeps the pool pass)."""
    from fedsim_amd import ops

    assert not ops.conv_pool_fusable((2, 32, 14, 14), 64, (5, 5), (1, 1), (1, 1, 1, 1),
                                     (2, 2, 2, 2, 1, 1))  # SimpleCNN conv2: chunked kernel
    assert not ops.conv_pool_fusable((2, 1, 28, 28), 32, (5, 5), (1, 1), (1, 1, 1, 1),
                                     (3, 3, 2, 2, 0, 0))  # not a 2 x 2 pool
    slab = torch.zeros(2, 64 * 32 * 25 + 64, device=DEV)
    with pytest.raises(ValueError):
        ops.teacher_conv2d(torch.zeros(2, 32, 14, 14, device=DEV), slab, 0, -1, 64, (5, 5),
                           (1, 1), (1, 1, 1, 1), shared=True, pool=(2, 2, 2, 2, 1, 1))


def test_simplecnn_replay_fuses_conv1_pool():
    """The reference's SimpleCNN (fedsim_amd.models restatement, Resize leaf
    included) replays with conv1's ReLU + max_pool2d(2, 2, padding=1) in the
    conv's store: one pool pass left (conv2's), outputs within fp32 rounding
    of each teacher's own forward."""
    from fedsim_amd import models
    from fedsim_amd.distributed.centralized.training import teacher_program as TP
    from fedsim_amd.utils import vector_to_named_parameters_like

    torch.manual_seed(21)
    model = models.SimpleCNN().to(DEV)
    named = list(model.named_parameters())
    base = torch.cat([p.detach().reshape(-1) for _, p in named])
    K = 12
    slab = torch.stack([base + 0.01 * torch.randn_like(base) for _ in range(K)])
    prog = TP.build(model, named, slab)
    assert prog is not None
    x = torch.randn(64, 1, 28, 28, device=DEV)
    got = prog(x)
    assert prog.fused_pools == 1 and prog.pool_launches == 1 and prog.conv_launches == 2
    want = torch.stack([functional_call(model, vector_to_named_parameters_like(slab[k], named),
                                        (x,)) for k in range(K)])
    err = float(torch.linalg.vector_norm((got - want).double()) /
                torch.linalg.vector_norm(want.double()))
    assert err <= 1e-5, err


def test_fused_relu_is_torch_relu_bitwise():
    """The ReLU fused into the Linear / Conv2d kernels is torch.relu's
    (x < 0 ? 0 : x): NaN stays NaN, so a teacher with non-finite outputs
    gives the reference's values (the kernels' fmaf chains start from +0, so
    their pre-activations are never -0)."""
    from fedsim_amd import ops

    g = torch.Generator(device=DEV).manual_seed(77)
    K, M, in_f, out_f = 3, 8, 5, 7
    slab = torch.randn(K, in_f * out_f + out_f, device=DEV, generator=g)
    slab[0, 0] = float("nan")                      # a NaN output column for teacher 0
    x = torch.randn(M, in_f, device=DEV, generator=g)
    plain = ops.teacher_linear(x, slab, 0, in_f * out_f, in_f, out_f, shared=True)
    fused = ops.teacher_linear(x, slab, 0, in_f * out_f, in_f, out_f, shared=True, relu=True)
    want = torch.relu(plain)
    assert torch.isnan(want).any()
    assert torch.equal(fused.view(torch.int32), want.view(torch.int32))
    C, OC = 1, 4
    cs = torch.randn(K, OC * C * 9 + OC, device=DEV, generator=g)
    cs[2, 0] = float("nan")
    xi = torch.randn(2, C, 6, 6, device=DEV, generator=g)
    plain = ops.teacher_conv2d(xi, cs, 0, OC * 9, OC, (3, 3), (1, 1), (1, 1, 1, 1), shared=True)
    fused = ops.teacher_conv2d(xi, cs, 0, OC * 9, OC, (3, 3), (1, 1), (1, 1, 1, 1), shared=True,
                               relu=True)
    want = torch.relu(plain)
    assert torch.isnan(want).any()
    assert torch.equal(fused.view(torch.int32), want.view(torch.int32))
