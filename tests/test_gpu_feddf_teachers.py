"""FedDF's teacher ensemble on the matrix cores (fedagg_teacher_linear_f32,
training/teacher_program.py): the layer kernel against an fp64 reference
within the f32 dot-product error bound, over ragged shapes; the traced replay
of whole models (MLP, CNN) over K stacked teachers against each teacher's own
forward; and the ensemble keeping the kernel path after its first-batch check.
Reference: fedsim/distributed/centralized/training/feddf.py:117-122."""
import numpy as np
import pytest
import torch
from torch.func import functional_call

from test_teacher_program import Cnn, Mlp, Tiny

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
                                       (Cnn, (64, 3, 8, 8))])
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
