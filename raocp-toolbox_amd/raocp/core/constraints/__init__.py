from .base_constraint import *
from .no_constraint import *
from .rectangle import *
