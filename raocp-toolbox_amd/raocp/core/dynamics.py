# SPDX-License-Identifier: Apache-2.0
# API restated from raocp-toolbox (Apache-2.0, Moran, Zhang, Sopasakis); see NOTICE.
"""Linear dynamics x+ = A x + B u (reference: raocp/core/dynamics.py:3-25)."""

__all__ = ["Dynamics"]


class Dynamics:
    """Pair (A, B); A is n_x-by-n_x, B is n_x-by-n_u. Rows must agree."""

    def __init__(self, state_dynamics, control_dynamics):
        if control_dynamics.shape[0] != state_dynamics.shape[0]:
            raise ValueError("Dynamics matrices rows are different sizes")
        self.__state_dynamics = state_dynamics
        self.__control_dynamics = control_dynamics

    @property
    def state_dynamics(self):
        """Matrix A."""
        return self.__state_dynamics

    @property
    def control_dynamics(self):
        """Matrix B."""
        return self.__control_dynamics
