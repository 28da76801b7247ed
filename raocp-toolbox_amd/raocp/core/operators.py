# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Linear operator L of the CP splitting and its adjoint (reference: raocp/core/operators.py:5-120).

`ell` / `ell_transpose` keep the reference's block-list calling convention: the
caller owns both lists, only the slots L (L^T) writes are replaced, every other
slot keeps what the caller passed. The arithmetic runs in HIP kernels through
`raocp_ell` / `raocp_ell_t`: the streaming MFMA wave tasks `k_ell3` / `k_ellt3`
(raocp_ell3.hip) on trees with uniform weight tables (and branching <= 4 for L^T), the
node-range block kernels `k_ell` / `k_ell_t` (raocp_kernels.hip) otherwise."""
import numpy as np

import raocp.core.cache as core_cache

__all__ = ["Operator"]


class Operator:
    def __init__(self, cache: core_cache.Cache):
        self.__cache = cache
        self.__raocp = cache.get_raocp()
        self.__num_nonleaf_nodes = int(self.__raocp.tree.num_nonleaf_nodes)
        self.__num_nodes = int(self.__raocp.tree.num_nodes)
        self.__segment_p = cache.get_primal_segments()
        self.__segment_d = cache.get_dual_segments()
        self.__native = cache.native

    @staticmethod
    def _flat(blocks):
        return np.concatenate([np.asarray(b, dtype=np.float64).reshape(-1) for b in blocks])

    def ell(self, input_primal, output_dual):
        """output_dual <- L(input_primal), operators.py:19-53."""
        out = self.__native.ell(self._flat(input_primal), template=self._flat(output_dual))
        blocks = self.__cache._blocks_d(out)
        for i, b in enumerate(blocks):
            output_dual[i] = b

    def ell_transpose(self, input_dual, output_primal):
        """output_primal <- L^T(input_dual), operators.py:55-94."""
        out = self.__native.ell_t(self._flat(input_dual), template=self._flat(output_primal))
        blocks = self.__cache._blocks_p(out)
        for i, b in enumerate(blocks):
            output_primal[i] = b

    def linop_ell(self, flat_primal):
        """(P,1) -> (D,1), zero template (operators.py:96-107)."""
        return self.__native.ell(np.asarray(flat_primal).reshape(-1)).reshape(-1, 1)

    def linop_ell_transpose(self, flat_dual):
        """(D,1) -> (P,1), zero template (operators.py:109-120)."""
        return self.__native.ell_t(np.asarray(flat_dual).reshape(-1)).reshape(-1, 1)
