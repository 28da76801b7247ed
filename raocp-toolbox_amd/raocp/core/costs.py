# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Quadratic stage/terminal cost (reference: raocp/core/costs.py:4-63).

The operator L only ever uses the matrix square roots; they are computed once
here with `scipy.linalg.sqrtm`, exactly as the reference does (costs.py:21,26),
so the per-mode tables uploaded to the GPU hold the same doubles.
"""
from scipy.linalg import sqrtm

__all__ = ["Quadratic"]


class Quadratic:
    """x'Qx (+ u'Ru for nonleaf nodes)."""

    def __init__(self, node_type, state_weights, control_weights=None):
        self.__node_type = node_type
        self._check_control_weights(control_weights)
        rows, cols = state_weights.shape[0], state_weights.shape[1]
        if rows != cols:
            raise Exception("Quadratic cost state weight matrix is not square")
        self.__state_weights = state_weights
        self.__sqrt_state_weights = sqrtm(state_weights)
        if control_weights is not None and control_weights.shape[0] != control_weights.shape[1]:
            raise Exception("Quadratic cost control weight matrix is not square")
        if node_type.is_nonleaf:
            self.__control_weights = control_weights
            self.__sqrt_control_weights = sqrtm(control_weights)
        elif not node_type.is_leaf:
            raise Exception("Control weights error in cost")

    def _check_control_weights(self, weights):
        nt = self.__node_type
        if nt.is_nonleaf and weights is None:
            raise Exception("No control weights provided for a nonleaf node")
        if nt.is_leaf and weights is not None:
            raise Exception("Control weights provided for a leaf node")

    @property
    def node_type(self):
        return self.__node_type

    @property
    def state_weights(self):
        return self.__state_weights

    @property
    def control_weights(self):
        return self.__control_weights

    @property
    def sqrt_state_weights(self):
        return self.__sqrt_state_weights

    @property
    def sqrt_control_weights(self):
        return self.__sqrt_control_weights

    def __repr__(self):
        return f"Cost item; type: {type(self).__name__}"

    __str__ = __repr__
