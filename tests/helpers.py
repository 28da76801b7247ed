"""Shared test helpers (problem construction from golden recipes, comparisons)."""
import numpy as np

from raocp.problems import build_problem, recipe_from_npz


def problem_from_golden(z, name):
    r = recipe_from_npz(z, name)
    tree, prob = build_problem(r)
    return r, tree, prob


def rel_err(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(np.max(np.abs(b)), 1e-300)
    return float(np.max(np.abs(a - b)) / scale) if a.size else 0.0


def trace_rel_err(a, b):
    a = np.atleast_2d(a)
    b = np.atleast_2d(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))
