"""MI355X-native SIMCA / VAE-SIMCA engine (host side of libocm.so)."""
import os

# HIP-graph replays of the VAE training step (ocm.vae_train) race in the ROCm
# 7.0 runtime's graph packet-capture path: with two replays in flight after a
# host sync the step reads half-updated state and the loss turns NaN within
# two replays (scripts/diag_vae_race2.py: 6/6 runs, 0/6 with this flag).  The
# runtime reads the flag once, at HIP initialisation, so it is set on import
# (before torch touches the GPU) unless the caller chose a value.
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from ._lib import OcmError, OcmNotConverged, load  # noqa: F401

__version__ = "0.1.0"
