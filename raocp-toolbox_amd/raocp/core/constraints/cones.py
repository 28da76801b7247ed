# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Convex cones and their projections (reference: raocp/core/constraints/cones.py:4-230).

Host-side (numpy) versions, kept for API parity and for callers that project
single vectors. Inside the CP loop the same projections are fused into the
`prox_gconj` HIP kernel (raocp_hip.hip): R_+ / {0}* element-wise, the second
order cone per child block and per leaf block.
"""
import numpy as np

__all__ = ["Real", "Zero", "NonnegativeOrthant", "SecondOrderCone", "Cartesian"]


def _check_dimension(cone_type, cone_dimension, vector):
    """Return the vector size; raise ValueError if a fixed cone dimension disagrees
    (cones.py:4-18)."""
    size = vector.size
    if cone_dimension is not None and cone_dimension != size:
        raise ValueError('%s cone dimension error: cone dimension = %d, input vector dimension = %d'
                         % (cone_type, cone_dimension, size))
    return size


class _Cone:
    def __init__(self, dimension=None):
        self._dim = dimension
        self._shape = None

    def _accept(self, vector):
        self._dim = _check_dimension(type(self), self._dim, vector)
        self._shape = vector.shape

    @property
    def dimension(self):
        """Cone dimension"""
        return self._dim


class Real(_Cone):
    """R^n; its dual is {0}."""

    def project(self, vector):
        self._accept(vector)
        return vector.copy()

    def project_onto_dual(self, vector):
        self._accept(vector)
        return np.zeros(self._dim).reshape(self._shape)


class Zero(_Cone):
    """{0}; its dual is R^n."""

    def project(self, vector):
        self._accept(vector)
        return np.zeros(self._dim).reshape(self._shape)

    def project_onto_dual(self, vector):
        self._accept(vector)
        return vector.copy()


class NonnegativeOrthant(_Cone):
    """R^n_+ (self dual)."""

    def project(self, vector):
        self._accept(vector)
        return np.maximum(vector, 0).astype(float).reshape(self._shape)

    def project_onto_dual(self, vector):
        return NonnegativeOrthant.project(self, vector)


class SecondOrderCone(_Cone):
    """{(f, t): ||f||_2 <= t} (self dual). Three cases, cones.py:113-132."""

    def project(self, vector):
        self._accept(vector)
        if self._dim < 3:
            raise Exception("Attempt to project a vector of size < 3 onto second order cone")
        t = vector[-1].reshape(1, 1)
        f = vector[0:-1]
        nf = np.linalg.norm(f)
        if nf <= t:
            return vector.copy()
        if nf <= -t:
            return np.zeros(shape=self._shape)
        scale = (nf + t) / 2
        return np.concatenate((scale * (f / nf), scale)).reshape(self._shape)

    def project_onto_dual(self, vector):
        return SecondOrderCone.project(self, vector)


class Cartesian:
    """Product of cones; a single stacked vector is split by the member dimensions."""

    def __init__(self, cones):
        self.__cones = cones
        self.__num_cones = len(cones)
        dims = [c.dimension for c in cones]
        self.__dimension = None if any(d is None for d in dims) else sum(dims)
        self.__dimensions = [None] * self.__num_cones

    def _apply(self, list_of_vectors, dual):
        parts = self._check_list_of_vectors(list_of_vectors)
        out = []
        for k, cone in enumerate(self.__cones):
            self.__dimensions[k] = _check_dimension(type(cone), cone.dimension, parts[k])
            out.append(cone.project_onto_dual(parts[k]) if dual else cone.project(parts[k]))
        self.__dimension = sum(self.__dimensions)
        return np.vstack(out) if len(list_of_vectors) == 1 else out

    def project(self, list_of_vectors):
        return self._apply(list_of_vectors, dual=False)

    def project_onto_dual(self, list_of_vectors):
        return self._apply(list_of_vectors, dual=True)

    def _check_list_of_vectors(self, list_of_vectors):
        if len(list_of_vectors) != 1:
            return list_of_vectors
        whole = list_of_vectors[0]
        parts, at = [], 0
        for cone in self.__cones:
            parts.append(whole[at: at + cone.dimension])
            at += cone.dimension
        return parts

    @property
    def types(self):
        return " x ".join(type(c).__name__ for c in self.__cones)

    @property
    def dimension(self):
        return self.__dimension

    @property
    def dimensions(self):
        return self.__dimensions

    @property
    def num_cones(self):
        return self.__num_cones
