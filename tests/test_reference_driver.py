"""The reference's own driver, unchanged, drives the drop-in.

/root/reference/scripts/run_optimization.py is imported AS IT IS from the reference checkout (never copied into this
repository, never sent to the GPU box; the test skips where the checkout is absent).  Its imports are satisfied the way a
maintainer's integration would:
  * ``optimization.Bayesian7.BayesianOptimizer``  -> the drop-in, bayesianoptimizer_amd.optimizer.BayesianOptimizer;
  * ``simulation.taichi.MPMSimulator``            -> a stub with the simulator's duck type (taichi is not installed and
                                                     opens a GUI, simulation/taichi.py:17), tests/stubs.py;
  * ``config.config``                             -> the reference's own module (imports cleanly).
The only other substitution is the drop-in's default engine factory (GPEngine needs a GPU): the CPU oracle engine.
run_optimization is then called with exactly the arguments of its signature (scripts/run_optimization.py:34-41) and
builds the optimizer with exactly its 10 keyword arguments (:116-127), the default GPConfig, the default acquisition and
test_csv_path="validation_set.csv" resolved against the reference checkout (the reference runs from its root).
"""
import importlib.util
import os
import sys
import types

import numpy as np
import pytest

REF = "/root/reference"
DRIVER = os.path.join(REF, "scripts", "run_optimization.py")

pytestmark = pytest.mark.skipif(not os.path.exists(DRIVER), reason="reference checkout not present (GPU box)")


@pytest.fixture
def reference_driver(monkeypatch):
    from bayesianoptimizer_amd import optimizer as dropin
    from tests.oracle_engine import OracleEngine
    from tests.stubs import StubSimulator

    constructed = []

    class MPMSimulator(StubSimulator):  # the reference's class name and constructor (simulation/taichi.py:21)
        def __init__(self, xml_path):
            super().__init__()
            self.xml_path = xml_path

    class RecordingOptimizer(dropin.BayesianOptimizer):
        def __init__(self, *args, **kwargs):
            constructed.append((args, dict(kwargs)))
            super().__init__(*args, **kwargs)
            constructed[-1] += (self,)

    sim_mod = types.ModuleType("simulation.taichi")
    sim_mod.MPMSimulator = MPMSimulator
    opt_mod = types.ModuleType("optimization.Bayesian7")
    opt_mod.BayesianOptimizer = RecordingOptimizer
    for name, mod in (("simulation", types.ModuleType("simulation")), ("simulation.taichi", sim_mod),
                      ("optimization", types.ModuleType("optimization")), ("optimization.Bayesian7", opt_mod)):
        monkeypatch.setitem(sys.modules, name, mod)
    monkeypatch.setattr(dropin, "GPEngine", lambda device=None: OracleEngine())
    monkeypatch.syspath_prepend(REF)  # config.config: the reference's own module
    monkeypatch.chdir(REF)            # the reference runs from its root: "validation_set.csv", "config/setting.xml"
    saved = {k: v for k, v in sys.modules.items() if k == "config" or k.startswith("config.")}
    spec = importlib.util.spec_from_file_location("reference_run_optimization", DRIVER)
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    yield module, constructed
    for k in [k for k in sys.modules if k == "config" or k.startswith("config.")]:
        if k not in saved:
            del sys.modules[k]


def _rows(path):
    with open(path) as fh:
        return sum(1 for _ in fh) - 1


def test_reference_run_optimization_drives_the_dropin_unchanged(reference_driver, tmp_path):
    module, constructed = reference_driver
    out = str(tmp_path / "results")
    best_params, best_value = module.run_optimization(total_evaluations=40, n_initial_points=24, batch_size=8, seed=0,
                                                      output_dir=out)
    csv = os.path.join(out, "optimization_results.csv")
    assert _rows(csv) == 40
    # exactly the 10 keyword arguments of scripts/run_optimization.py:116-127, nothing positional
    args, kwargs, opt = constructed[0]
    assert args == ()
    # the default GPConfig: hyperparameters by marginal likelihood, one set per output (the multi-output SingleTaskGP)
    assert opt.gp_model.independent and opt.engine.calls.get("mll", 0) > 0
    assert len({tuple(p.lengthscales(5)) for p in opt.gp_model.params}) > 1
    assert sorted(kwargs) == sorted(["simulator", "bounds_list", "output_dir", "n_initial_points", "n_batches",
                                     "batch_size", "svgp_threshold", "resume", "target_total", "test_csv_path"])
    assert kwargs["n_initial_points"] == 24 and kwargs["n_batches"] == 2 and kwargs["resume"] is False
    assert kwargs["test_csv_path"] == "validation_set.csv" and kwargs["target_total"] == 40
    assert kwargs["simulator"].cleaned  # the driver's finally: simulator.cleanup() (:131-134)
    assert best_params.shape == (5,) and np.isfinite(best_value)
    # the relative test set resolved as the reference expects: 20,000 validation rows scored every round
    log = os.path.join(out, "validation_log.csv")
    assert any(",Test_Set," in line for line in open(log))
    # resume: the driver counts the CSV lines and asks for the 8 missing evaluations
    module.run_optimization(total_evaluations=48, n_initial_points=24, batch_size=8, seed=0, output_dir=out)
    args, kwargs, _ = constructed[1]
    assert kwargs["resume"] is True and kwargs["n_initial_points"] == 0 and kwargs["n_batches"] == 1
    assert _rows(csv) == 48
    data = np.loadtxt(csv, delimiter=",", skiprows=1)
    lo = np.array([b[0] for b in kwargs["bounds_list"]])
    hi = np.array([b[1] for b in kwargs["bounds_list"]])
    assert np.all(data[:, :5] >= lo - 1e-9) and np.all(data[:, :5] <= hi + 1e-9)
    # a third call at the same target does nothing (run_optimization.py:73-76)
    assert module.run_optimization(total_evaluations=48, n_initial_points=24, batch_size=8, seed=0,
                                   output_dir=out) == (None, None)
    assert len(constructed) == 2
