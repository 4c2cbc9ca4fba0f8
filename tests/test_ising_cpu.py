"""Ising MF-Q: the numpy oracle and the host-side stream generator against the reference fixtures.

tests/golden/ising_*.npz were recorded by running the reference Scenario (Ising.py) and world
(core.py) under main_MFQ_Ising.py's loop.  CPU only."""
import json
import os
import sys

import numpy as np
import pytest

import common

sys.path.insert(0, os.path.join(common.REPO, "oracle"))
import ising_oracle  # noqa: E402

with open(os.path.join(common.GOLDEN, "ising_manifest.json")) as f:
    CASES = json.load(f)["cases"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_trajectory(name):
    c = CASES[name]
    fx = np.load(os.path.join(common.GOLDEN, name + ".npz"))
    out = ising_oracle.mfq(c["n_agents"], c["temperature"], c["steps"], lr=c["lr"], act_rate=c["act_rate"],
                           seed=c["seed"])
    assert out["steps"] == c["stopped_after"]
    np.testing.assert_array_equal(out["actions"], fx["actions"])
    assert out["order"].tobytes() == fx["order"].tobytes()
    np.testing.assert_array_equal(out["n_up"], fx["n_up"])
    assert out["q"].tobytes() == fx["q_final"].tobytes()          # bit-exact float64 Q table


def test_neighbour_table_matches_oracle():
    from mfrl_amd.ising import neighbour_table
    for n in (16, 100, 400, 900):
        np.testing.assert_array_equal(neighbour_table(n), ising_oracle.neighbours(n))


def test_reference_stream_reproduces_initial_spins_and_first_actions():
    from mfrl_amd.ising import reference_stream
    c = CASES["ising20_t08"]
    fx = np.load(os.path.join(common.GOLDEN, "ising20_t08.npz"))
    spins0, u, mask = reference_stream(c["seed"], c["n_agents"], 5, c["act_rate"])
    np.testing.assert_array_equal(spins0, fx["spins0"])
    # step 0: Q == 0 -> p = [0.5, 0.5] -> action = (u >= 0.5)
    np.testing.assert_array_equal((u[0] >= 0.5).astype(np.int8), fx["actions"][0])
    assert (mask == 0xFFFFFFFF).all() or c["n_agents"] % 32 != 0


def test_dropin_examples_wins_over_a_namespace_examples(tmp_path):
    """main_MFQ_Ising.py sits next to the reference's namespace package `examples/`; the drop-in's
    regular `examples` package must still be the one `examples.ising_model` resolves to."""
    import subprocess
    import sys
    shadow = tmp_path / "examples" / "ising_model"
    shadow.mkdir(parents=True)
    (shadow / "__init__.py").write_text("raise ImportError('the namespace portion was imported')\n")
    code = ("import sys; sys.path.insert(0, %r); import examples.ising_model as m; print(m.__file__)"
            % str(tmp_path))
    env = dict(os.environ, PYTHONPATH=common.PY_DIR)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().startswith(common.PY_DIR), out.stdout


def test_oracle_episodes_match_reference_fixture():
    """main_MFQ_Ising.py -epi 3 (tests/golden/ising4_epi3.npz): the episodes run in sequence on one
    numpy stream; the first two stop early, so the third starts from draws shifted by both stops."""
    import ising_oracle
    with open(os.path.join(common.GOLDEN, "ising_manifest.json")) as f:
        c = json.load(f)["episode_cases"]["ising4_epi3"]
    fx = np.load(os.path.join(common.GOLDEN, "ising4_epi3.npz"))
    got = ising_oracle.mfq_episodes(c["n_agents"], c["temperature"], c["steps"], c["episodes"], seed=c["seed"])
    for k, ep in enumerate(got):
        p = "e%d_" % k
        assert ep["steps"] == int(fx[p + "stop"]) == c["stops"][k]
        np.testing.assert_array_equal(ep["actions"], fx[p + "actions"])
        assert ep["order"].tobytes() == fx[p + "order"].tobytes()
        np.testing.assert_array_equal(ep["n_up"], fx[p + "n_up"])
        assert ep["q"].tobytes() == fx[p + "q_final"].tobytes()


@pytest.mark.parametrize("n,steps", [(100, 40), (400, 6)])
def test_per_agent_loop_restatement_matches_the_vectorised_oracle(n, steps):
    """oracle.ising_oracle.mfq_loop (the CPU baseline of the reference's per-agent loop) consumes the same numpy
    stream and gives the same Q table and order parameters as the vectorised oracle, bit for bit."""
    import ising_oracle
    a = ising_oracle.mfq_loop(n, 0.8, steps, seed=13)
    b = ising_oracle.mfq(n, 0.8, steps, seed=13)
    assert a["steps"] == b["steps"]
    assert a["q"].tobytes() == b["q"].tobytes()
    assert a["order"].tobytes() == b["order"].tobytes()


@pytest.mark.parametrize("seed,n,k", [(13, 400, 400), (21, 100, 50), (5, 16, 3)])
def test_numpy_stream_model(seed, n, k):
    """The consumption model the device stream follows (csrc/ising_kernels.hip k_mt_words / k_ising_scan), restated
    word by word in oracle/ising_oracle.py MT19937Words, against numpy's own legacy RandomState: the seeding, the
    choice(2) spins, random_sample's doubles and choice(N, k, replace=False)'s shuffle draws, over two steps."""
    rs, mt = np.random.RandomState(seed), ising_oracle.MT19937Words(seed)
    assert list(rs.get_state()[1]) == mt.key
    assert [int(rs.choice(2)) for _ in range(2 * n)] == [mt.choice2() for _ in range(2 * n)]
    for _ in range(2):
        assert rs.random_sample(n).tobytes() == np.array([mt.random_sample() for _ in range(n)]).tobytes()
        assert list(rs.choice(n, k, replace=False)) == mt.choice_no_replace(n, k)
    assert rs.randint(0, 2 ** 32, dtype=np.uint64) == mt.word()
