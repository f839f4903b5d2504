"""Network registry resolved by ConfigParser.init_obj('network', module_network, ...)
(reference model/network.py).  The denoisers on the north-star path: UNetModified2 and DiffWave."""
from .UNetModified2 import UNetModified2  # noqa: F401
from .diffwave import DiffWave  # noqa: F401
