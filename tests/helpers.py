"""Shared test helpers: tolerances, seeded inputs, oracle <-> device conversion."""
import numpy as np
import torch

# BASELINE.json north star: outputs within 1e-3 relative of the reference path.
REL_TOL = 1e-3


def rel_inf(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def rel_l2(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.norm().item()
    return (a - b).norm().item() / (den if den > 0 else 1.0)


def rng_tensor(shape, seed, scale=1.0, lo=None, hi=None):
    r = np.random.default_rng(seed)
    if lo is not None:
        v = r.uniform(lo, hi, size=shape)
    else:
        v = r.standard_normal(shape) * scale
    return torch.tensor(v, dtype=torch.float32)


def dev(t):
    return t.to("cuda").contiguous()


def f64(t):
    return t.detach().cpu().double()
