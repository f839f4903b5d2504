"""Network registry resolved by ConfigParser.init_obj('network', module_network, ...)
(reference model/network.py).  The denoisers on the north-star path: UNetModified2, DiffWave and
WaveGrad."""
from .UNetModified2 import UNetModified2  # noqa: F401
from .diffwave import DiffWave  # noqa: F401
from .wavegrad import WaveGrad  # noqa: F401
