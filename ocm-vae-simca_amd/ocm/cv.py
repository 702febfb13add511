"""Fold engine for class-wise SIMCA cross-validation (filled in below)."""


def grid(base_est, X, y, cv, lv_values, param_grid, class_index, store_predictions):
    return None, None
