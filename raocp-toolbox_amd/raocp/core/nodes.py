# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Node-type tags (reference: raocp/core/nodes.py:3-31).

`Nonleaf()` / `Leaf()` instances are passed to costs and constraints to say
which part of the scenario tree they apply to.
"""

__all__ = ["Node", "Nonleaf", "Leaf"]


class Node:
    """Untyped node tag: neither nonleaf nor leaf."""
    _NONLEAF = False
    _LEAF = False

    @property
    def is_nonleaf(self):
        return self._NONLEAF

    @property
    def is_leaf(self):
        return self._LEAF


class Nonleaf(Node):
    """Tag for nodes at stages 0..N-1 (they carry a control and children)."""
    _NONLEAF = True


class Leaf(Node):
    """Tag for nodes at the final stage N."""
    _LEAF = True
