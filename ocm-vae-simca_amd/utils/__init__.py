"""Drop-in replacement for the reference's ``utils`` package
(TEAM-AIOLY/OCM-VAE-SIMCA utils/__init__.py:1-9): put
``ocm-vae-simca_amd/`` on ``sys.path`` and ``from utils import SIMCA`` runs
the MI355X engine."""
from .SIMCA import SIMCA
from .CVSIMCA import (
    cross_validate_simca_grid,
    plot_cv,
    ClasswiseKFoldWithExternalVal,
)
from .data_utils import object_aware_splits

__all__ = ["SIMCA", "cross_validate_simca_grid", "plot_cv", "ClasswiseKFoldWithExternalVal", "object_aware_splits"]
