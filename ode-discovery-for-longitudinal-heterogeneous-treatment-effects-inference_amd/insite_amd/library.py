"""Candidate library Theta(x, u) descriptors — the pysindy ``PolynomialLibrary`` surface used by
the reference (``libs_m/ct/src/models/sindy.py:185-188``), expressed as an exponent table.

A library over the inputs ``[x0, u0, .., u{U-1}]`` (one state, U static covariates) is the int8
table ``exps[F, 1+U]``; column j evaluates ``x0**exps[j,0] * prod_i u_i**exps[j,1+i]``.  The joint
("one ODE") model puts ``n_inputs`` per-step treatment inputs first among the u's (the reference's
``U = concat(treatments, statics)``, pkpd/utils.py:488-497): ``exps[F, 1 + n_inputs + n_statics]``.  Column
order follows pysindy: bias, linear terms, then products by degree in ``itertools.combinations``
(interaction_only) or ``combinations_with_replacement`` order.  The GPU kernels receive this table
through the C ABI (``insite_gram_f64`` / ``insite_rollout_f64``).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class PolyLibrary:
    exps: np.ndarray          # int8 [F, 1 + n_inputs + n_statics]
    input_names: tuple        # ('x0', 'u0', 'u1')
    n_inputs: int = 0         # per-step treatment inputs (joint model), between x0 and the statics

    @property
    def n_terms(self) -> int:
        return int(self.exps.shape[0])

    @property
    def n_statics(self) -> int:
        return int(self.exps.shape[1]) - 1 - self.n_inputs

    @property
    def state_degree(self) -> int:
        return int(self.exps[:, 0].max())

    def get_feature_names(self) -> list:
        """pysindy-style names: '1', 'x0', 'x0 u0', 'x0^2', ..."""
        names = []
        for e in self.exps:
            parts = []
            for i, k in enumerate(e):
                if k == 1:
                    parts.append(self.input_names[i])
                elif k > 1:
                    parts.append(f"{self.input_names[i]}^{int(k)}")
            names.append(" ".join(parts) if parts else "1")
        return names

    def ctypes_table(self) -> np.ndarray:
        """Contiguous int8 copy handed to the C ABI (built once per library object)."""
        t = self.__dict__.get("_table")
        if t is None:
            t = np.ascontiguousarray(self.exps, dtype=np.int8)
            t.setflags(write=False)
            object.__setattr__(self, "_table", t)
        return t


def polynomial_library(n_statics: int, degree: int = 2, interaction_only: bool = True,
                       include_bias: bool = True, state_name: str = "x0", n_inputs: int = 0) -> PolyLibrary:
    n_in = 1 + int(n_inputs) + int(n_statics)
    comb = itertools.combinations if interaction_only else itertools.combinations_with_replacement
    rows = []
    for deg in range(0 if include_bias else 1, degree + 1):
        for c in comb(range(n_in), deg):
            e = [0] * n_in
            for i in c:
                e[i] += 1
            rows.append(e)
    names = (state_name,) + tuple(f"u{i}" for i in range(int(n_inputs) + int(n_statics)))
    return PolyLibrary(np.array(rows, dtype=np.int8), names, int(n_inputs))
