"""File formats and helper extensions around the PH engine (``mpisppy/utils``)."""
