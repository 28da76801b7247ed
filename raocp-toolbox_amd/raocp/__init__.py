"""raocp (MI355X-native build).

Drop-in replacement for smokinmirror/raocp-toolbox's Python package
(`/root/reference/raocp/__init__.py:1-2`): the builder API (`raocp.core.RAOCP`,
`MarkovChainScenarioTreeFactory`, costs/risks/constraints) is kept, while the
Chambolle-Pock inner loop (`Operator.ell/ell_transpose`, `Cache` prox operators,
`Solver.chock`) runs in hand-written HIP kernels for gfx950 behind the C-ABI
library `libraocp_hip.so` (see `include/raocp_hip.h`).
"""
import raocp.core.constraints
import raocp.core
