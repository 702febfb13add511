"""MI355X-native SIMCA / VAE-SIMCA engine (host side of libocm.so)."""
import os

# HIP-graph replays of the VAE training step (ocm.vae_train) race in the ROCm
# 7.0 runtime's graph packet-capture path: with two replays in flight after a
# host sync the step reads half-updated state and the loss turns NaN within
# two replays (scripts/diag_vae_race2.py: 6/6 runs, 0/6 with this flag).  The
# runtime reads the flag once, at HIP initialisation, so it is set on import
# (before torch touches the GPU) unless the caller chose a value.
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

# The graphed DDP step waits, before capturing, until ProcessGroupNCCL's
# watchdogs have retired the caller's eager collectives; it reads that from
# their flight recorder (ocm/rccl.py), which torch keeps only with a non-zero
# buffer size, read when the process group starts.  A bounded ring of 2000
# entries unless the caller chose a size.
if not any(v in os.environ for v in ("TORCH_FR_BUFFER_SIZE", "TORCH_NCCL_TRACE_BUFFER_SIZE")):
    os.environ["TORCH_FR_BUFFER_SIZE"] = "2000"

from ._lib import OcmError, OcmNotConverged, load  # noqa: F401

__version__ = "0.1.0"
