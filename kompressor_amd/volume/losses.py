"""Volume losses -- ``src/kompressor/volume/losses.py`` (off the hot path)."""

from ..losses import mean_squared_error, mean_abs_error, mean_charbonnier_error, total_variation  # noqa: F401


def mean_total_variation(input):
    """volume/losses.py:30-35 -- mean of the signed z, y, x forward differences, / 3."""
    return total_variation(input, (1, 2, 3))
