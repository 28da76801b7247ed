# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""AVaR risk measure as a conic ambiguity set (reference: raocp/core/risks.py:5-82).

For a nonleaf node with c children and conditional probabilities p:
    E = [alpha I; -I; 1'],  F = (2c+1)x0,  cone = R_+^{2c} x {0},  b = [p; 0; 1].
The GPU path only needs alpha and p (the kernel-space projection has a closed
form in alpha), the matrices are kept for API parity.
"""
import numpy as np
import raocp.core.constraints.cones as core_cones

__all__ = ["AVaR"]


class AVaR:
    def __init__(self, alpha):
        if not 0 <= alpha <= 1:
            raise ValueError("alpha value '%d' not supported" % alpha)
        self.__alpha = alpha
        self.__num_children = None
        self.__children_probabilities = None
        self.__matrix_e = None
        self.__matrix_f = None
        self.__cone = None
        self.__vector_b = None

    def _make_e_f_cone_b(self):
        c = self.__num_children
        ident = np.eye(c)
        self.__matrix_e = np.concatenate((self.__alpha * ident, -ident, np.ones((1, c))), axis=0)
        self.__matrix_f = np.zeros((2 * c + 1, 0))
        self.__cone = core_cones.Cartesian([core_cones.NonnegativeOrthant(dimension=2 * c),
                                            core_cones.Zero(dimension=1)])
        p = np.asarray(self.__children_probabilities).reshape(-1, 1)
        self.__vector_b = np.concatenate((p, np.zeros((c, 1)), np.ones((1, 1))), axis=0)

    @property
    def is_risk(self):
        return True

    @property
    def alpha(self):
        return self.__alpha

    @property
    def matrix_e(self):
        return self.__matrix_e

    @property
    def matrix_f(self):
        return self.__matrix_f

    @property
    def cone(self):
        return self.__cone

    @property
    def vector_b(self):
        return self.__vector_b

    @property
    def probs(self):
        return self.__children_probabilities

    @probs.setter
    def probs(self, vector):
        self.__children_probabilities = vector
        self.__num_children = vector.size
        self._make_e_f_cone_b()

    def __repr__(self):
        return f"Risk item; type: {type(self).__name__}, alpha: {self.__alpha}; cone: {self.__cone.types}"

    __str__ = __repr__
