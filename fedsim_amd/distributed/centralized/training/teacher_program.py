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
* every ``nn.Conv2d`` (groups 1, dilation 1, zero padding) is one implicit-GEMM
  launch for all K teachers (``fedagg_teacher_conv2d_f32``:
  v_mfma_f32_32x32x2_f32, the im2col gathered into LDS, never stored), a
  following ReLU fused;
* every chain of zero ``F.pad`` / ``local_response_norm`` / ``max_pool2d``
  after it (the reference's SimpleCNN / SimpleCNN2, simple_models.py:156-159,
  245-252) is one pass (``fedagg_pad_lrn_maxpool_f32``);
* each maximal run of the other nodes between them (reshapes, other layers)
  is ONE ``torch.vmap`` over the teacher dimension; a run that does not
  depend on the teachers (the input's own preprocessing) runs once, unbatched.
  A conv or pool node whose runtime shapes the kernels do not take runs the
  same way.

A parameterless module from outside ``torch.nn`` (torchvision's ``Resize``
at the head of every reference model, simple_models.py:47,107,195, whose
forward branches on the input's shape) is traced as one leaf call rather than
into; on the input it runs once per batch, unbatched.

``build`` returns None when the model does not trace (``build_or_reason``
also says why), so the caller keeps its whole-model ``vmap`` path; the
ensemble also checks the replay against that path on its first batch before
using it, and counts and reports every fallback (feddf.py TeacherEnsemble).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import nn
from torch.fx.node import map_arg
from torch.func import functional_call

from .... import ops

F = torch.nn.functional
_RELU_FUNCS = (torch.relu, F.relu)
# graph nodes whose value is random: a forward that has one is not a pure
# function of (teacher, input), so its outputs may not be reused
_RANDOM_FUNCS = {F.dropout, F.dropout1d, F.dropout2d, F.dropout3d, F.alpha_dropout,
                 F.feature_alpha_dropout, torch.dropout, torch.rand, torch.randn,
                 torch.rand_like, torch.randn_like, torch.randint, torch.randint_like,
                 torch.randperm, torch.bernoulli, torch.normal, torch.multinomial,
                 torch.poisson}
_RANDOM_METHODS = {"normal_", "uniform_", "bernoulli_", "random_", "exponential_",
                   "geometric_", "log_normal_", "cauchy_"}


class _Tracer(torch.fx.Tracer):
    """torch.fx's default tracer, except that a module with no parameters
    and no buffers from outside ``torch.nn`` is one leaf call."""

    def is_leaf_module(self, m: nn.Module, qualname: str) -> bool:
        if super().is_leaf_module(m, qualname):
            return True
        return (not type(m).__module__.startswith("torch.")
                and next(m.parameters(), None) is None and next(m.buffers(), None) is None)


def _trace(model: nn.Module) -> torch.fx.GraphModule:
    tracer = _Tracer()
    graph = tracer.trace(model)
    return torch.fx.GraphModule(tracer.root, graph, type(model).__name__)


def _bind(node, names, defaults):
    """The node's arguments after its input, by name (positional, then
    keyword, then the defaults); None when it passes unknown ones."""
    vals = dict(defaults)
    if len(node.args) - 1 > len(names):
        return None
    for n, v in zip(names, node.args[1:]):
        vals[n] = v
    for n, v in node.kwargs.items():
        if n not in names:
            return None
        vals[n] = v
    if any(isinstance(v, torch.fx.Node) for v in vals.values()) or any(
            n not in vals for n in names):
        return None
    return vals


def _pair(v):
    return (int(v[0]), int(v[1])) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _pool_item(node, modules):
    """("pad", (top, bottom, left, right)) / ("lrn", (size, alpha, beta, k)) /
    ("pool", (kh, kw, sh, sw, ph, pw)) for a node fedagg_pad_lrn_maxpool_f32
    can run, else None."""
    if node.op == "call_function" and node.target is F.pad:
        a = _bind(node, ("pad", "mode", "value"), {"mode": "constant", "value": None})
        if a is None or a["mode"] != "constant" or a["value"] not in (None, 0, 0.0):
            return None
        pad = a["pad"]
        if not isinstance(pad, (tuple, list)) or len(pad) not in (2, 4) or any(
                not isinstance(v, int) or v < 0 for v in pad):
            return None
        pad = tuple(pad) + (0, 0) * (len(pad) == 2)
        return ("pad", (pad[2], pad[3], pad[0], pad[1]))
    if node.op == "call_function" and node.target is F.local_response_norm:
        a = _bind(node, ("size", "alpha", "beta", "k"), {"alpha": 1e-4, "beta": 0.75, "k": 1.0})
        if a is None or not isinstance(a["size"], int) or a["size"] <= 0:
            return None
        return ("lrn", (a["size"], float(a["alpha"]), float(a["beta"]), float(a["k"])))
    if node.op == "call_function" and node.target is F.max_pool2d:
        a = _bind(node, ("kernel_size", "stride", "padding", "dilation", "ceil_mode",
                         "return_indices"),
                  {"stride": None, "padding": 0, "dilation": 1, "ceil_mode": False,
                   "return_indices": False})
    elif node.op == "call_module" and len(node.args) == 1 and not node.kwargs:
        mod = modules.get(node.target)
        if type(mod) is nn.MaxPool2d:
            a = dict(kernel_size=mod.kernel_size, stride=mod.stride, padding=mod.padding,
                     dilation=mod.dilation, ceil_mode=mod.ceil_mode,
                     return_indices=mod.return_indices)
        elif type(mod) is nn.LocalResponseNorm:
            return ("lrn", (int(mod.size), float(mod.alpha), float(mod.beta), float(mod.k)))
        elif type(mod) in (nn.ZeroPad2d, nn.ConstantPad2d) and getattr(mod, "value", 0) == 0:
            l, r, t, b = mod.padding
            return ("pad", (t, b, l, r))
        else:
            return None
    else:
        return None
    if a is None or a["ceil_mode"] or a["return_indices"] or _pair(a["dilation"]) != (1, 1):
        return None
    kh, kw = _pair(a["kernel_size"])
    sh, sw = _pair(a["stride"]) if a["stride"] not in (None, (), []) else (kh, kw)
    ph, pw = _pair(a["padding"])
    return ("pool", (kh, kw, sh, sw, ph, pw))


def _conv_geometry(mod):
    """(kernel, stride, (top, bottom, left, right)) of an nn.Conv2d the conv
    kernel runs (groups 1, dilation 1, zero padding), else None."""
    if (type(mod) is not nn.Conv2d or mod.groups != 1 or tuple(mod.dilation) != (1, 1)
            or mod.padding_mode != "zeros"):
        return None
    if isinstance(mod.padding, str):
        l, r, t, b = ((0, 0, 0, 0) if mod.padding == "valid"
                      else tuple(mod._reversed_padding_repeated_twice))
    else:
        t = b = int(mod.padding[0])
        l = r = int(mod.padding[1])
    return tuple(mod.kernel_size), tuple(mod.stride), (t, b, l, r)


def _is_relu(node, modules) -> bool:
    if node.op == "call_function" and node.target in _RELU_FUNCS:
        return not node.kwargs.get("inplace", False) and len(node.args) == 1
    if node.op == "call_method" and node.target == "relu":
        return len(node.args) == 1
    if node.op == "call_module":
        return type(modules.get(node.target)) is nn.ReLU
    return False


class _Segment(object):
    """A run of graph nodes replayed by one vmap (kind "ops"), one Linear or
    Conv2d layer on the matrix cores (kind "linear" / "conv"), or one
    pad / LRN / max-pool chain (kind "pool")."""

    __slots__ = ("kind", "nodes", "inputs", "outputs", "params", "fn", "spec", "pool_next")

    def __init__(self, kind, nodes, spec=None):
        self.kind = kind
        self.nodes = nodes
        self.inputs: List = []   # nodes outside the run that it reads
        self.outputs: List = []  # nodes of the run read after it
        self.params: List = []   # parameter names the run reads
        self.fn = None           # the run as generated code (kind "ops"; the
        #                          fallback of "conv" / "pool")
        self.spec = spec         # conv geometry / pool chain
        self.pool_next = None    # conv: the 2 x 2 / 2 max-pool segment its store may fuse


class TeacherProgram(object):
    """``program(x)`` = the K teachers' outputs on input ``x``, [K, ...]."""

    def __init__(self, model: nn.Module, named, slab: torch.Tensor, impl=None):
        # impl: TEST HOOK replacing the ops module (its teacher_linear /
        # teacher_conv2d / pad_lrn_maxpool, same signatures), so the graph
        # replay can be checked on the CPU
        self.impl = ops if impl is None else impl
        self.gm = _trace(model)
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
        # a ReLU whose input is a Linear / Conv2d node used only by it: fused
        self.fused = set()
        self.alias = {}
        for node in nodes:
            if _is_relu(node, self.modules):
                src = node.args[0]
                if (isinstance(src, torch.fx.Node) and (self._is_linear(src) or self._is_conv(src))
                        and len(src.users) == 1):
                    self.fused.add(src)
                    self.alias[node] = src
        self.segments = self._partition(nodes)
        self.linear_launches = 0
        self.conv_launches = 0
        self.pool_launches = 0
        self.fused_pools = 0  # pool segments run inside the conv's store

    @property
    def has_random_ops(self) -> bool:
        """Whether the traced forward draws random numbers (dropout, rand ...),
        outside of leaf modules (train-mode ``nn.Dropout`` modules are the
        caller's check, feddf._pure_forward)."""
        for node in self.gm.graph.nodes:
            if node.op == "call_function" and node.target in _RANDOM_FUNCS:
                return True
            if node.op == "call_method" and node.target in _RANDOM_METHODS:
                return True
        return False

    def _is_linear(self, node) -> bool:
        return (node.op == "call_module" and type(self.modules.get(node.target)) is nn.Linear
                and len(node.args) == 1 and not node.kwargs)

    def _is_conv(self, node) -> bool:
        return (node.op == "call_module" and len(node.args) == 1 and not node.kwargs
                and _conv_geometry(self.modules.get(node.target)) is not None)

    def _pool_chain(self, node):
        """The longest chain from ``node`` of pads, at most one LRN and at
        most one max pool (ending it), each node feeding only the next:
        (nodes, pads, lrn, pool), or None."""
        nodes, pads, lrn, pool = [], [0, 0, 0, 0], None, None
        cur = node
        while True:
            item = _pool_item(cur, self.modules)
            if item is None or (item[0] == "lrn" and lrn is not None):
                break
            nodes.append(cur)
            if item[0] == "pad":
                pads = [p + q for p, q in zip(pads, item[1])]
            elif item[0] == "lrn":
                lrn = item[1]
            else:
                pool = item[1]
                break
            users = list(cur.users)
            if len(users) != 1 or not users[0].args or users[0].args[0] is not cur:
                break
            cur = users[0]
        if not nodes:
            return None
        return nodes, tuple(pads), lrn, pool

    def _partition(self, nodes):
        segs = []
        run = []
        taken = set()

        def special(seg):
            nonlocal run
            if run:
                segs.append(_Segment("ops", run))
                run = []
            segs.append(seg)

        for node in nodes:
            if node.op in ("placeholder", "output") or node in self.alias or node in taken:
                continue
            if self._is_linear(node):
                special(_Segment("linear", [node]))
            elif self._is_conv(node):
                special(_Segment("conv", [node], _conv_geometry(self.modules[node.target])))
            else:
                chain = self._pool_chain(node)
                if chain is not None:
                    taken.update(chain[0])
                    special(_Segment("pool", chain[0], chain[1:]))
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
            if seg.kind in ("ops", "conv", "pool"):
                seg.fn = self._compile(seg)
        for a, b in zip(segs, segs[1:]):
            if a.kind == "conv" and b.kind == "pool" and self._pool_fusable(a, b):
                a.pool_next = b
        return segs

    def _pool_fusable(self, conv, pool) -> bool:
        """A max pool of 2 x 2 / stride 2 (padding 0 or 1; no pad, no LRN)
        that is the only reader of the conv's (ReLU'd) output: candidates for
        the conv kernel's pooled store (checked against the runtime shape)."""
        pads, lrn, spec = pool.spec
        if pads != (0, 0, 0, 0) or lrn is not None or spec is None:
            return False
        kh, kw, sh, sw, ph, pw = spec
        if (kh, kw, sh, sw) != (2, 2, 2, 2) or ph != pw or ph not in (0, 1):
            return False
        node = conv.nodes[0]
        head = pool.nodes[0]
        out = [u for u in node.users]
        if len(out) == 1 and out[0] in self.alias:  # the fused ReLU in between
            out = list(out[0].users)
        return out == [head] and pool.inputs == [node]

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
        y = self.impl.teacher_linear(x, self.slab, w, b, mod.in_features, mod.out_features,
                                     shared=not batched, relu=node in self.fused)
        self.linear_launches += 1
        return y.view(self.K, *lead, mod.out_features)

    def _conv(self, seg, env, done) -> bool:
        """The conv node on the matrix cores; False when its runtime input is
        not the 4-D (per teacher) f32 image batch the kernel takes.  With a
        fusable max pool after it (SimpleCNN's conv1 -> relu -> max_pool2d(2,
        2, padding=1)) the pool runs in the conv's store and its segment is
        added to ``done``."""
        node = seg.nodes[0]
        v, batched = env[seg.inputs[0]]
        if (not isinstance(v, torch.Tensor) or v.dtype != torch.float32
                or v.dim() != (5 if batched else 4)):
            return False
        mod = self.modules[node.target]
        kernel, stride, pads = seg.spec
        w = self.offs[node.target + ".weight"][0]
        b = self.offs[node.target + ".bias"][0] if mod.bias is not None else -1
        pool = None
        nxt = seg.pool_next
        fusable = getattr(self.impl, "conv_pool_fusable", None)
        if nxt is not None and fusable is not None and fusable(
                v.shape, mod.out_channels, kernel, stride, pads, nxt.spec[2]):
            pool = nxt.spec[2]
        y = self.impl.teacher_conv2d(v.contiguous(), self.slab, w, b, mod.out_channels, kernel,
                                     stride, pads, shared=not batched, relu=node in self.fused,
                                     pool=pool)
        self.conv_launches += 1
        if pool is None:
            env[node] = (y, True)
        else:
            self.fused_pools += 1
            env[nxt.nodes[-1]] = (y, True)
            done.add(nxt)
        return True

    def _pool(self, seg, env) -> bool:
        """The pad / LRN / max-pool chain in one pass; False when its runtime
        input is not a 4-D (per teacher) f32 image batch the kernel takes."""
        v, batched = env[seg.inputs[0]]
        if (not isinstance(v, torch.Tensor) or v.dtype != torch.float32
                or v.dim() != (5 if batched else 4)):
            return False
        pads, lrn, pool = seg.spec
        try:  # ValueError: a shape the kernel does not take (checked before any launch)
            y = self.impl.pad_lrn_maxpool(v.contiguous(), pads, lrn, pool)
        except ValueError:
            return False
        self.pool_launches += 1
        env[seg.nodes[-1]] = (y, batched)
        return True

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
            if o in self.fused:  # a conv run here: its fused ReLU is not in the run's code
                v = torch.relu(v)
            env[o] = (v, True)

    # teachers per replay pass: bounds the activations (SimpleCNN2's first
    # conv output is 9.4 MB per teacher per 64-sample batch)
    max_teachers = 512

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if self.K <= self.max_teachers:
            return self._replay(x)
        full, K = self.slab, self.K
        step = -(-K // -(-K // self.max_teachers))
        outs = []
        try:
            for k0 in range(0, K, step):
                self.slab = full[k0:k0 + step]
                self.K = self.slab.shape[0]
                outs.append(self._replay(x))
        finally:
            self.slab, self.K = full, K
        return torch.cat(outs)

    def _replay(self, x: torch.Tensor) -> torch.Tensor:
        env = {p: (x, False) for p in self.placeholders}
        done = set()  # pool segments already run by a conv's pooled store
        for seg in self.segments:
            if seg in done:
                continue
            if seg.kind == "linear":
                node = seg.nodes[0]
                v, b = env[self.alias.get(node.args[0], node.args[0])]
                env[node] = (self._linear(node, v, b), True)
            elif seg.kind == "conv" and self._conv(seg, env, done):
                pass
            elif seg.kind == "pool" and self._pool(seg, env):
                pass
            else:
                self._run_ops(seg, env)
        res = self.output.args[0]
        v, b = env[self.alias.get(res, res)]
        if not b or not isinstance(v, torch.Tensor):
            raise NotImplementedError("the model's output does not depend on its weights")
        return v


def build_or_reason(model: nn.Module, named, slab: torch.Tensor,
                    impl=None) -> Tuple[Optional[TeacherProgram], Optional[str]]:
    """(TeacherProgram, None), or (None, why not): its forward does not trace,
    uses parameters outside its own ``named_parameters`` layout, or has no
    Linear / Conv2d layer for the matrix cores to run."""
    try:
        prog = TeacherProgram(model, named, slab, impl)
    except Exception as e:  # noqa: BLE001 - untraceable forward: the caller keeps vmap
        return None, f"the forward does not trace ({type(e).__name__}: {e})"
    if not any(s.kind in ("linear", "conv") for s in prog.segments):
        return None, "the forward has no nn.Linear / nn.Conv2d layer to replay"
    return prog, None


def build(model: nn.Module, named, slab: torch.Tensor, impl=None) -> Optional[TeacherProgram]:
    """A TeacherProgram for ``model``, or None (see ``build_or_reason``)."""
    return build_or_reason(model, named, slab, impl)[0]
