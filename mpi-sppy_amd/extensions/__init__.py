"""PH extensions (hook objects called from the PH loop; ``mpisppy/extensions``)."""
