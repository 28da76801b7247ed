# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Box constraint lo <= [x; u] <= hi (reference: raocp/core/constraints/rectangle.py:5-69).

The GPU prox of g* clips with the same bounds (`raocp_hip.h`, box tables).
A NaN reaching the clip raises ValueError in the reference (rectangle.py:50-59);
the device path reports it through the context's NaN flag (status code
RAOCP_ERR_NAN_IN_BOX) and the Python shim re-raises the same ValueError.
"""
import numpy as np
import raocp.core.constraints.base_constraint as bc

__all__ = ["Rectangle"]


class Rectangle(bc.Constraint):
    def __init__(self, node_type, _min, _max):
        super().__init__(node_type)
        self._check_constraints(_min, _max)
        self.__min = _min
        self.__max = _max

    @property
    def is_active(self):
        return True

    @property
    def lower(self):
        """Lower bounds (flattened); used by the device packer."""
        return self.__min

    @property
    def upper(self):
        return self.__max

    def _set_matrices(self):
        nx, nu = self.state_size, self.control_size
        self.state_matrix = np.concatenate((np.eye(nx), np.zeros((nu, nx))), axis=0)
        if self.node_type.is_nonleaf:
            self.control_matrix = np.concatenate((np.zeros((nx, nu)), np.eye(nu)), axis=0)

    def project(self, vector):
        self._check_input(vector)
        out = np.zeros(vector.shape)
        for i in range(vector.size):
            out[i] = self._constrain(vector[i], self.__min[i], self.__max[i])
        return out

    @staticmethod
    def _check_constraints(_min, _max):
        if _min.size != _max.size:
            raise Exception("Rectangle constraint - min and max vectors sizes are not equal")
        for lo, hi in zip(_min.reshape(-1), _max.reshape(-1)):
            if lo is None and hi is None:
                raise Exception("Rectangle constraint - both min and max constraints cannot be None")
            if lo is not None and hi is not None and lo > hi:
                raise Exception("Rectangle constraint - min greater than max")

    @staticmethod
    def _constrain(value, mini, maxi):
        if mini <= value <= maxi:
            return value
        if value <= mini:
            return mini
        if value >= maxi:
            return maxi
        raise ValueError(f"Rectangle constraint - '{value}' value cannot be constrained")

    def _check_input(self, vector):
        if vector.size != self.state_matrix.shape[0]:
            raise Exception("Rectangle constraint - input vector does not equal expected size")

    def __repr__(self):
        return f"Constraint; type: {type(self).__name__}"

    __str__ = __repr__
