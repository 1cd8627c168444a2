"""Solver-plugin boundary of the engine (``mpisppy/spopt.py:876-913``: ``SolverFactory(solver_name)``
per subproblem): the ``phg`` plugin over the C ABI (:mod:`.phg`) and the standard-form extractor
that turns a model into the CSR arrays the ABI takes (:mod:`.extract`)."""
from .extract import StandardForm, as_scenario_model, extract, to_linear_model  # noqa: F401
from .phg import PHGSolver, SolverFactory, register_solver  # noqa: F401
