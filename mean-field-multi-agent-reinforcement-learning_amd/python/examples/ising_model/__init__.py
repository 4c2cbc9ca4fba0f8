"""Drop-in of the reference examples/ising_model package, backed by the HIP Ising lattice.

``examples.ising_model.load('Ising.py').Scenario()`` returns this package's Scenario (the name
is resolved next to this file, as the reference's imp.load_source does -- __init__.py:5-7)."""
import importlib.util
import os.path as osp


def load(name):
    path = osp.join(osp.dirname(__file__), name)
    spec = importlib.util.spec_from_file_location("ising_scenario_" + osp.splitext(osp.basename(name))[0], path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod
