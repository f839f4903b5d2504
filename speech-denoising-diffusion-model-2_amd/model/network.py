"""Network registry resolved by ConfigParser.init_obj('network', module_network, ...)
(reference model/network.py).  Only the denoisers on the north-star path are provided."""
from .UNetModified2 import UNetModified2  # noqa: F401
