"""mpisppy_amd -- MI355X-native Progressive Hedging engine (drop-in for mpi-sppy's PH hot path)."""
__version__ = "0.1.0"
