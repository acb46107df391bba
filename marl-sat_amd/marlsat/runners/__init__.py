"""Training / evaluation drivers (src/runners of the reference)."""
