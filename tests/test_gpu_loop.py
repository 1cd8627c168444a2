"""GPU: the pipelined PH iteration (PHBase.update_and_solve) against the sequential one at the loop's
exits -- a time limit tripping mid-run (the drained conv must stay in conv_history) and
the PHIterLimit exit -- on farmer cm=10, 30 scenarios.  The time limit is made deterministic by
patching PHBase._time_over to trip at a given iteration."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def _run(pipeline, trip_at=None, limit=12):
    opts = {"solver_name": "phg", "PHIterLimit": limit, "defaultPHrho": 1.0, "convthresh": 1e-10,
            "verbose": False, "display_progress": False, "pdhg_pipeline": pipeline,
            "time_limit": 1e9 if trip_at else None}
    ph = PH(opts, farmer.scenario_names_creator(30), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": 30})
    if trip_at:
        ph._time_over = lambda: ph._PHIter >= trip_at
    ph.ph_main(finalize=False)
    return ph


@pytest.mark.parametrize("trip_at", [None, 1, 2, 5])
def test_pipelined_exits_match_sequential(trip_at):
    a, b = _run(True, trip_at), _run(False, trip_at)
    assert a._PHIter == b._PHIter
    assert len(a.conv_history) == len(b.conv_history) == a._PHIter
    np.testing.assert_allclose(a.conv_history, b.conv_history, rtol=1e-12)
    np.testing.assert_array_equal(a.Ws(), b.Ws())
    np.testing.assert_array_equal(a.nonants(), b.nonants())
    np.testing.assert_array_equal(a.xbars(), b.xbars())
