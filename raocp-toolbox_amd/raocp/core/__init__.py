"""Public namespace of raocp.core — same names as the reference
(`/root/reference/raocp/core/__init__.py:1-10`)."""
from .nodes import *
from .scenario_tree import *
from .raocp_spec import *
from .costs import *
from raocp.core.constraints.cones import *
from .risks import *
from .operators import *
from .cache import *
from .solver import *
