# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Constraint base class (reference: raocp/core/constraints/base_constraint.py:4-118).

A constraint on node variables is written as  Gamma_x x + Gamma_u u  in a set C.
Subclasses fill the selector matrices in `_set_matrices` once both sizes are
known; the transposes are cached because L^T applies them.
"""
import numpy as np

__all__ = ["Constraint"]


class Constraint:
    def __init__(self, node_type):
        self.__node_type = node_type
        self.__state_size = None
        self.__control_size = None
        self.__state_matrix = None
        self.__control_matrix = None
        self.__state_matrix_transposed = None
        self.__control_matrix_transposed = None

    def project(self, vector):
        return None

    # ----- getters
    @property
    def is_active(self):
        raise Exception("Base constraint accessed - actual constraint must not be setup")

    @property
    def node_type(self):
        return self.__node_type

    @property
    def state_size(self):
        return self.__state_size

    @property
    def control_size(self):
        return self.__control_size

    @property
    def state_matrix(self):
        return self.__state_matrix

    @property
    def control_matrix(self):
        return self.__control_matrix

    @property
    def state_matrix_transposed(self):
        if self.__state_matrix_transposed is None:
            raise Exception("Constraint state matrix transpose called but is None")
        return self.__state_matrix_transposed

    @property
    def control_matrix_transposed(self):
        if self.__control_matrix_transposed is None:
            raise Exception("Constraint control matrix transpose called but is None")
        return self.__control_matrix_transposed

    # ----- setters
    def _refresh(self):
        self._set_matrices()
        self._get_transpose()

    @state_size.setter
    def state_size(self, size):
        self.__state_size = size
        nt = self.__node_type
        if nt.is_nonleaf:
            if self.__control_size is not None:
                self._refresh()
        elif nt.is_leaf:
            self.__control_size = 0
            self._refresh()
        else:
            raise Exception("Node type missing")

    @control_size.setter
    def control_size(self, size):
        self.__control_size = size
        nt = self.__node_type
        if nt.is_nonleaf:
            if self.__state_size is not None:
                self._refresh()
        elif nt.is_leaf:
            raise Exception("Attempt to set control size on leaf node")
        else:
            raise Exception("Node type missing")

    def _set_matrices(self):
        return None

    def _get_transpose(self):
        nt = self.__node_type
        if nt.is_nonleaf:
            self.__state_matrix_transposed = np.transpose(self.state_matrix)
            self.__control_matrix_transposed = np.transpose(self.control_matrix)
        elif nt.is_leaf:
            self.__state_matrix_transposed = np.transpose(self.state_matrix)
        else:
            raise Exception("Node type missing")

    @state_matrix.setter
    def state_matrix(self, matrix):
        self.__state_matrix = matrix

    @control_matrix.setter
    def control_matrix(self, matrix):
        nt = self.__node_type
        if nt.is_nonleaf:
            self.__control_matrix = matrix
        elif nt.is_leaf:
            raise Exception("Attempt to set control constraint matrix of leaf node")
        else:
            raise Exception("Node type missing")

    def __repr__(self):
        return "Base constraint"

    __str__ = __repr__
