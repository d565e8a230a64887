"""Glue between the reference-style Python functions and the layer-program executor.

`run_net(kind, builder, x, is_training)` resolves the variable scope (variables.variable_scope),
builds or fetches the compiled NetProgram for the input shape, and runs it through an autograd
Function: outputs flow back through the hand-scheduled HIP backward; parameter gradients accumulate
into the ParamChunk's flat gradient buffer (read them with `chunk.grad_view(name)`).
"""
import torch

from . import variables
from .program import NetProgram, NetRun

_PROGRAMS = {}


def get_program(net_scope, builder, H, W, cin, **kw):
    prefix = "/".join(p for p in (variables.current_prefix(), net_scope) if p)
    key = (prefix, builder.__name__, H, W, cin, tuple(sorted(kw.items())))
    prog = _PROGRAMS.get(key)
    if prog is None:
        spec = builder(H, W, cin, scope=net_scope, **kw)
        specs, bn = spec.param_specs()
        chunk = variables.get_store().get_or_create(prefix, specs, bn, variables.current_reuse())
        if not hasattr(chunk, "anchor"):
            chunk.anchor = torch.zeros(1, device="cuda", dtype=torch.float32, requires_grad=True)
        prog = NetProgram(spec, chunk)
        _PROGRAMS[key] = prog
    return prog


def clear_programs():
    _PROGRAMS.clear()


class _NetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, x, prog, is_training):
        run = NetRun(prog, x.shape[0])
        outs = prog.forward(run, x.detach(), is_training)
        ctx.run, ctx.prog = run, prog
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        need_x = ctx.needs_input_grad[1]
        dx = ctx.prog.backward(ctx.run, list(grads), need_input_grad=need_x)
        return None, (dx.contiguous() if dx is not None else None), None, None


def run_net(net_scope, builder, x, is_training=True, **kw):
    if x.dim() != 4:
        raise ValueError(f"expected NHWC image batch, got {tuple(x.shape)}")
    if x.dtype != torch.float32 or not x.is_cuda:
        raise ValueError("inputs must be float32 tensors on the GPU (the HIP path has no CPU fallback)")
    N, H, W, C = x.shape
    prog = get_program(net_scope, builder, H, W, C, **kw)
    outs = _NetFunction.apply(prog.chunk.anchor, x, prog, is_training)
    return list(outs), prog
