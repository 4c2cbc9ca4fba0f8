"""The C oracle (oracle/battle_oracle.c) against the reference-recorded golden fixtures.

These pin the oracle: every observable output of every step (view/feature bytes, ids,
rewards, alive flags, post-step positions, counts, done) must be bit-identical to what
the reference engine produced on the same placements and actions.  CPU only."""
import os
import subprocess

import numpy as np
import pytest

import common


@pytest.fixture(scope="module", autouse=True)
def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(common.REPO, "oracle")], check=True)


@pytest.mark.parametrize("name", ["battle40_seq", "battle40_s1", "battle40_s2", "battle64"])
def test_oracle_replays_reference(name):
    assert common.replay_case(common.ORACLE_LIB, name) == []


@pytest.mark.slow
def test_oracle_replays_reference_large_map():
    assert common.replay_case(common.ORACLE_LIB, "battle256") == []


def test_oracle_full_observation_tensors():
    fx = np.load(os.path.join(common.GOLDEN, "battle40_seq.npz"))
    case = common.manifest()["cases"]["battle40_seq"]
    env, handles = common.battle_env(common.ORACLE_LIB, 40)
    env.reset()
    for g, pos in common.placement_for(case, case["episodes"][0]):
        env.add_agents(handles[g], method="custom", pos=pos)
    for g in range(2):
        v, f = env.get_observation(handles[g])
        np.testing.assert_array_equal(v, fx["e0_view_s0_g%d" % g])
        np.testing.assert_array_equal(f, fx["e0_feat_s0_g%d" % g])


def test_oracle_edge_case_nan_minimap():
    import edge_case
    edge_case.check(common.ORACLE_LIB)


@pytest.mark.parametrize("name", ["battle256_seq"])
def test_oracle_replays_reference_full_large_episodes(name):
    """256x256, 2048 per side: two full 400-step episodes in one env (band-mode move order on the
    thinned late-game map, clear_dead churn, the attack-shuffle LCG carried across the restart)."""
    assert common.replay_case(common.ORACLE_LIB, name) == []


@pytest.mark.parametrize("name,lanes", [("battle256_rollout", (512, 512)), ("battle64_rollout", (64, 256)),
                                        ("battle64_rollout", (64, 512))])
def test_oracle_replays_reference_rollout_fixture(name, lanes):
    """Env 0 of the 256x256 / 64x64 bench batch under the device rush policy (restated on the host), two
    episodes, on the C oracle: every step equals the reference recording (tests/golden/battle*_rollout), with
    the episode returns summed in each engine's team orders (k_rollout 64 / 256, the few-env stepper 64 / 512,
    the large-env queue kernel 512)."""
    import rollout_check as rck
    fx = rck.RolloutFixture(name, lanes)
    c = fx.case
    rep = rck.EnvReplay(c["map_size"], fx.placement, c["env"], c["n_envs"], c["max_steps"], True, c["seed"], c["eps"],
                        "k_rollout_bigq", lanes=lanes)
    for t in range(c["steps"]):
        rep.advance(t + 1)
        bad = fx.compare(rck.replay_records(rep), 0, t)
        assert not bad, bad[:8]
