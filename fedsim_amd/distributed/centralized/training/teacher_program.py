"""FedDF's K teacher forwards as one graph over the stacked teachers.

The reference runs every client model on each distillation batch, one after
another (fedsim/distributed/centralized/training/feddf.py:117-122).  Here the
server model's forward is traced once (torch.fx) and replayed over all K
teachers at once, with the teachers' parameters read straight from the [K, P]
slab of their flat vectors (parameters_to_vector layout):

* every ``nn.Linear`` node runs on the matrix cores for all K teachers in one
  launch (``fedagg_teacher_linear_f32``: v_mfma_f32_16x16x4_f32, each
  teacher's weights read once per 64 samples), with a following ReLU fused
  into its epilogue;
* each maximal run of the other nodes between them (convolutions, pooling,
  normalisation, reshapes) is ONE ``torch.vmap`` over the teacher dimension,
  so the convolutional part costs what the whole-model ``vmap`` costs; a run
  that does not depend on the teachers (the input's own preprocessing) runs
  once, unbatched.

``build`` returns None when the model does not trace, so the caller keeps
its whole-model ``vmap`` path; the ensemble also checks the replay against
that path on its first batch before using it (feddf.py TeacherEnsemble).
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn
from torch.fx.node import map_arg
from torch.func import functional_call

from .... import ops

_RELU_FUNCS = (torch.relu, torch.nn.functional.relu)


def _is_relu(node, modules) -> bool:
    if node.op == "call_function" and node.target in _RELU_FUNCS:
        return not node.kwargs.get("inplace", False) and len(node.args) == 1
    if node.op == "call_method" and node.target == "relu":
        return len(node.args) == 1
    if node.op == "call_module":
        return type(modules.get(node.target)) is nn.ReLU
    return False


class _Segment(object):
    """A run of graph nodes replayed by one vmap (kind "ops") or one Linear
    layer on the matrix cores (kind "linear")."""

    __slots__ = ("kind", "nodes", "inputs", "outputs", "params", "fn")

    def __init__(self, kind, nodes):
        self.kind = kind
        self.nodes = nodes
        self.inputs: List = []   # nodes outside the run that it reads
        self.outputs: List = []  # nodes of the run read after it
        self.params: List = []   # parameter names the run reads
        self.fn = None           # the run as generated code (kind "ops")


class TeacherProgram(object):
    """``program(x)`` = the K teachers' outputs on input ``x``, [K, ...]."""

    def __init__(self, model: nn.Module, named, slab: torch.Tensor, linear=None):
        # linear: TEST HOOK replacing ops.teacher_linear (same signature), so
        # the graph replay can be checked on the CPU
        self.linear_impl = ops.teacher_linear if linear is None else linear
        self.gm = torch.fx.symbolic_trace(model)
        self.modules = dict(self.gm.named_modules())
        self.slab = slab
        self.K = slab.shape[0]
        self.offs = {}
        off = 0
        for name, p in named:
            self.offs[name] = (off, p.numel(), tuple(p.shape))
            off += p.numel()
        nodes = list(self.gm.graph.nodes)
        self.placeholders = [n for n in nodes if n.op == "placeholder"]
        self.output = [n for n in nodes if n.op == "output"][0]
        # a ReLU whose input is a Linear node used only by it: fused
        self.fused = set()
        self.alias = {}
        for node in nodes:
            if _is_relu(node, self.modules):
                src = node.args[0]
                if (src.op == "call_module" and type(self.modules.get(src.target)) is nn.Linear
                        and len(src.users) == 1):
                    self.fused.add(src)
                    self.alias[node] = src
        self.segments = self._partition(nodes)
        self.linear_launches = 0

    def _is_linear(self, node) -> bool:
        return (node.op == "call_module" and type(self.modules.get(node.target)) is nn.Linear
                and len(node.args) == 1 and not node.kwargs)

    def _partition(self, nodes):
        segs = []
        run = []
        for node in nodes:
            if node.op in ("placeholder", "output") or node in self.alias:
                continue
            if self._is_linear(node):
                if run:
                    segs.append(_Segment("ops", run))
                    run = []
                segs.append(_Segment("linear", [node]))
            else:
                run.append(node)
        if run:
            segs.append(_Segment("ops", run))
        resolve = lambda n: self.alias.get(n, n)  # noqa: E731
        for seg in segs:
            inside = set(seg.nodes)
            ins = []
            for node in seg.nodes:
                for a in node.all_input_nodes:
                    a = resolve(a)
                    if a not in inside and a not in ins:
                        ins.append(a)
                if node.op == "call_module" and not self._is_linear(node):
                    mod = self.modules[node.target]
                    seg.params += [node.target + "." + n for n, _ in mod.named_parameters()]
                elif node.op == "get_attr" and node.target in self.offs:
                    seg.params.append(node.target)
            seg.inputs = ins
            for node in seg.nodes:
                users = [u for u in node.users]
                users += [uu for u in node.users if u in self.alias for uu in u.users]
                if any(u not in inside and u not in self.alias for u in users):
                    seg.outputs.append(node)
        for name in (p for s in segs for p in s.params):
            if name not in self.offs:
                raise KeyError(f"parameter {name} is not in the flat vector layout")
        for seg in segs:
            if seg.kind == "ops":
                seg.fn = self._compile(seg)
        return segs

    def _compile(self, seg) -> torch.fx.GraphModule:
        """The run as generated Python (fx codegen): fn(*inputs, *params)
        returns the run's outputs; modules with parameters are called through
        functional_call on the per-teacher parameter arguments."""
        g = torch.fx.Graph()
        env = {}
        for i, n in enumerate(seg.inputs):
            env[n] = g.placeholder(f"in_{i}")
        pnodes = {name: g.placeholder(f"p_{j}") for j, name in enumerate(seg.params)}
        remap = lambda n: env[self.alias.get(n, n)]  # noqa: E731
        for node in seg.nodes:
            if node.op == "call_module" and any(True for _ in
                                                self.modules[node.target].parameters()):
                mod = self.modules[node.target]
                ps = {n: pnodes[node.target + "." + n] for n, _ in mod.named_parameters()}
                env[node] = g.call_function(
                    functional_call,
                    (g.get_attr(node.target), ps, tuple(map_arg(node.args, remap)),
                     dict(map_arg(node.kwargs, remap))))
            elif node.op == "get_attr" and node.target in pnodes:
                env[node] = pnodes[node.target]
            else:
                env[node] = g.node_copy(node, remap)
        g.output(tuple(env[o] for o in seg.outputs))
        return torch.fx.GraphModule(self.gm, g)

    def _param(self, name: str) -> torch.Tensor:
        off, n, shape = self.offs[name]
        return self.slab[:, off:off + n].view(self.K, *shape)

    def _linear(self, node, value, batched):
        mod = self.modules[node.target]
        w = self.offs[node.target + ".weight"][0]
        b = self.offs[node.target + ".bias"][0] if mod.bias is not None else -1
        x = value.contiguous().float()
        lead = x.shape[1:-1] if batched else x.shape[:-1]
        y = self.linear_impl(x, self.slab, w, b, mod.in_features, mod.out_features,
                             shared=not batched, relu=node in self.fused)
        self.linear_launches += 1
        return y.view(self.K, *lead, mod.out_features)

    def _run_ops(self, seg, env):
        vals = [env[n][0] for n in seg.inputs]
        dims = [0 if env[n][1] else None for n in seg.inputs]
        pvals = [self._param(p) for p in seg.params]
        if not pvals and not any(d == 0 for d in dims):  # independent of the teachers
            outs = seg.fn(*vals)
            for o, v in zip(seg.outputs, outs):
                env[o] = (v, False)
            return
        outs = torch.vmap(seg.fn, in_dims=tuple(dims) + (0,) * len(pvals))(*vals, *pvals)
        for o, v in zip(seg.outputs, outs):
            if not isinstance(v, torch.Tensor):
                raise NotImplementedError("a non-tensor value crosses a Linear layer")
            env[o] = (v, True)

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        env = {p: (x, False) for p in self.placeholders}
        for seg in self.segments:
            if seg.kind == "linear":
                node = seg.nodes[0]
                v, b = env[self.alias.get(node.args[0], node.args[0])]
                env[node] = (self._linear(node, v, b), True)
            else:
                self._run_ops(seg, env)
        res = self.output.args[0]
        v, b = env[self.alias.get(res, res)]
        if not b or not isinstance(v, torch.Tensor):
            raise NotImplementedError("the model's output does not depend on its weights")
        return v


def build(model: nn.Module, named, slab: torch.Tensor, linear=None) -> Optional[TeacherProgram]:
    """A TeacherProgram for ``model``, or None when its forward does not trace,
    uses parameters outside its own ``named_parameters`` layout, or has no
    Linear layer for the matrix cores to run."""
    try:
        prog = TeacherProgram(model, named, slab, linear)
    except Exception:  # noqa: BLE001 - untraceable forward: the caller keeps vmap
        return None
    if not any(s.kind == "linear" for s in prog.segments):
        return None
    return prog
