# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""The inactive constraint (reference: raocp/core/constraints/no_constraint.py:4-13).
Loaded on every node by `RAOCP`; its dual slots (eta_7 / eta_14) stay placeholders."""
import raocp.core.constraints.base_constraint as bc

__all__ = ["No"]


class No(bc.Constraint):
    def __init__(self, node_type=None):
        super().__init__(node_type)

    @property
    def is_active(self):
        return False
