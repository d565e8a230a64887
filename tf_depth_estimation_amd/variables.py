"""Model variables with TF-1 names and shapes, stored flat in HBM.

Mirrors the reference's variable handling (`tf.variable_scope(...)` + `scope.reuse_variables()`,
train_depth_then_cam_lr.py:123-154) and its checkpoint contract: every
variable keeps its TF name (`model/depth_net/cnv1/weights`) and TF layout (conv [kh,kw,cin,cout],
deconv [kh,kw,cout,cin]).  MI355X-first layout: all trainable variables of one network live in ONE
16-byte-aligned flat fp32 buffer (`ParamChunk.flat`) with a matching flat gradient buffer and Adam
slots, so the optimizer is a single HBM-streaming launch and the data-parallel gradient all-reduce is
one contiguous RCCL buffer.  BN moving statistics (model variables, not trainable) live in a
separate flat buffer.

Initialisation follows slim's defaults (Glorot-uniform weights, zero biases/beta, moving mean 0 /
variance 1) with a per-variable PCG64 stream keyed by (seed, crc32(name)), so values do not depend on
creation order.
"""
import contextlib
import zlib

import numpy as np
import torch


def glorot_uniform(rng, shape):
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    fan_in, fan_out = rf * shape[-2], rf * shape[-1]
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape)


class ParamChunk:
    """Flat storage for the trainable variables and BN statistics of one network instance."""

    def __init__(self, specs, bn_specs, device="cuda", seed=1):
        # specs: list of (name, shape, init in {'glorot','zeros'}); bn_specs: list of (name, C)
        self.offsets, self.shapes = {}, {}
        off = 0
        for name, shape, _ in specs:
            n = int(np.prod(shape))
            self.offsets[name], self.shapes[name] = off, tuple(shape)
            off += (n + 3) // 4 * 4
        self.numel = off
        host = np.zeros(off, dtype=np.float32)
        for name, shape, init in specs:
            if init == "glorot":
                rng = np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))
                v = glorot_uniform(rng, shape).astype(np.float32)
                o = self.offsets[name]
                host[o:o + v.size] = v.reshape(-1)
        self.flat = torch.from_numpy(host).to(device)
        self.grad = torch.zeros_like(self.flat)
        self.adam_m = torch.zeros_like(self.flat)
        self.adam_v = torch.zeros_like(self.flat)
        # BN moving statistics: [mean(C) | var(C)] per layer
        self.bn_offsets = {}
        boff = 0
        for name, c in bn_specs:
            self.bn_offsets[name] = (boff, c)
            boff += 2 * ((c + 3) // 4 * 4)
        bn_host = np.zeros(max(boff, 4), dtype=np.float32)
        for name, (o, c) in self.bn_offsets.items():
            cp = (c + 3) // 4 * 4
            bn_host[o + cp:o + cp + c] = 1.0
        self.bn = torch.from_numpy(bn_host).to(device)

    def view(self, name):
        o = self.offsets[name]
        shape = self.shapes[name]
        return self.flat[o:o + int(np.prod(shape))].view(shape)

    def grad_view(self, name):
        o = self.offsets[name]
        shape = self.shapes[name]
        return self.grad[o:o + int(np.prod(shape))].view(shape)

    def moving(self, bn_name):
        o, c = self.bn_offsets[bn_name]
        cp = (c + 3) // 4 * 4
        return self.bn[o:o + c], self.bn[o + cp:o + cp + c]

    def names(self):
        return list(self.offsets.keys())

    def state_dict(self):
        """TF-named tensors (trainable variables + BN moving statistics), checkpoint contract."""
        out = {n: self.view(n) for n in self.offsets}
        for bn_name in self.bn_offsets:
            m, v = self.moving(bn_name)
            out[bn_name + "/moving_mean"] = m
            out[bn_name + "/moving_variance"] = v
        return out

    def load_state_dict(self, sd, strict=True):
        with torch.no_grad():
            for n in self.offsets:
                if n in sd:
                    self.view(n).copy_(torch.as_tensor(sd[n]).reshape(self.shapes[n]))
                elif strict:
                    raise KeyError(n)
            for bn_name in self.bn_offsets:
                m, v = self.moving(bn_name)
                if bn_name + "/moving_mean" in sd:
                    m.copy_(torch.as_tensor(sd[bn_name + "/moving_mean"]))
                    v.copy_(torch.as_tensor(sd[bn_name + "/moving_variance"]))
                elif strict:
                    raise KeyError(bn_name)


class VariableStore:
    """Process-wide store of ParamChunks keyed by the variable-scope prefix of the net instance."""

    def __init__(self):
        self.chunks = {}
        self.seed = 1

    def get_or_create(self, prefix, specs, bn_specs, reuse):
        if prefix in self.chunks:
            ch = self.chunks[prefix]
            if reuse is False:
                raise ValueError(f"Variable {prefix}/... already exists, disallowed (reuse=False)")
            return ch
        if reuse is True:
            raise ValueError(f"Variable {prefix}/... does not exist, and reuse=True")
        ch = ParamChunk([(f"{prefix}/{n}", s, i) for n, s, i in specs],
                        [(f"{prefix}/{n}", c) for n, c in bn_specs], seed=self.seed)
        ch.prefix = prefix
        self.chunks[prefix] = ch
        return ch

    def reset(self, seed=1):
        self.chunks = {}
        self.seed = seed


_STORE = VariableStore()
_SCOPE = []   # stack of (name, reuse)


def get_store():
    return _STORE


@contextlib.contextmanager
def variable_scope(name, reuse=None):
    """tf.variable_scope analogue: nets called inside create (or, under reuse, share) variables
    named `<scope>/<net scope>/<layer>/...`."""
    _SCOPE.append([name, reuse])
    try:
        yield _ScopeHandle(len(_SCOPE) - 1)
    finally:
        _SCOPE.pop()


class _ScopeHandle:
    def __init__(self, idx):
        self.idx = idx

    def reuse_variables(self):
        _SCOPE[self.idx][1] = True


def current_prefix():
    return "/".join(s[0] for s in _SCOPE if s[0])


def current_reuse():
    for _, r in reversed(_SCOPE):
        if r is not None:
            return r
    return None
