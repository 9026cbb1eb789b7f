"""Image losses -- ``src/kompressor/image/losses.py`` (off the hot path)."""

from ..losses import mean_squared_error, mean_abs_error, mean_charbonnier_error, total_variation  # noqa: F401


def mean_total_variation(input):
    """image/losses.py:30-34 -- mean of the signed y, x forward differences, / 2."""
    return total_variation(input, (1, 2))
