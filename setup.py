from setuptools import setup

setup(
    name="mpisppy_amd",
    version="0.1.0",
    description="MI355X-native Progressive Hedging engine (drop-in for the mpi-sppy PH hot path)",
    packages=["mpisppy_amd", "mpisppy_amd.examples"],
    package_dir={"mpisppy_amd": "mpi-sppy_amd"},
    package_data={"mpisppy_amd": ["libphg.so", "csrc/*"]},
)
