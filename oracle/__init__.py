"""oracle/ -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).

CPU restatement of the reference PH hot path (maxfey/mpi-sppy @ 2024-12-20):

* ``highs``  -- one HiGHS 1.8.0 solve per scenario (scipy's bundled copy), standing in for the
  Pyomo ``SolverFactory`` plugin called at ``mpisppy/spopt.py:184-231``.
* ``models`` -- Pyomo-free restatements of the reference example generators
  (``examples/farmer/farmer.py``, ``mpisppy/tests/examples/farmer.py``, ``examples/hydro/hydro.py``,
  ``examples/sslp``, ``examples/netdes``) in standard form.
* ``ph``     -- numpy restatement of ``PHBase``/``SPOpt``/``SPBase`` semantics
  (``mpisppy/phbase.py:32-112,301-371,829-1061``; ``mpisppy/spopt.py:99-497``;
  ``mpisppy/spbase.py:188-220,297-395,509-526``; ``mpisppy/utils/sputils.py:790-856``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline.  The product (``mpi-sppy_amd/``) never
imports it.

Parity pinning: the restatement is pinned against the reference's own known-answer fixtures
(``mpisppy/tests/examples/w_test_data/{w_file,xbar_file}.csv``; farmer EF objective -108390;
farmer-30 trivial bound -137846; hydro trivial bound 180 / E[obj] 190) -- see
``tests/test_oracle_pins.py``.  The reference itself cannot be imported here (``pyomo`` and
``mpi4py`` are absent; an ordinary ImportError, not a permission denial).
"""
