"""MI355X-native SIMCA / VAE-SIMCA engine (host side of libocm.so)."""
from ._lib import OcmError, OcmNotConverged, load  # noqa: F401

__version__ = "0.1.0"
