"""The C oracle against the reference engine build itself (oracle/_ref, when it is built)
on randomized scenarios: random walls and 'random' placements (engine LCG), duplicate
custom placements, uneven groups, two episodes per env (LCG persistence).  CPU only."""
import os

import pytest

import common
from test_battle_gpu import _random_scenario

pytestmark = pytest.mark.skipif(not os.path.exists(common.REF_LIB), reason="oracle/_ref not built")


@pytest.mark.parametrize("map_size,n0,n1,seed,walls", [
    (12, 5, 9, 1, 6), (20, 30, 30, 2, 20), (33, 60, 40, 3, 50), (64, 128, 128, 4, 0), (110, 300, 250, 5, 100)])
def test_oracle_matches_reference_random_scenarios(map_size, n0, n1, seed, walls):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    ref = _random_scenario(common.REF_LIB, map_size, n0, n1, seed, 60, walls, episodes=2)
    got = _random_scenario(common.ORACLE_LIB, map_size, n0, n1, seed, 60, walls, episodes=2)
    assert len(got) == len(ref)
    first_bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if a != b), None)
    assert first_bad is None, "first divergence at step %s" % first_bad


def test_oracle_matches_reference_large_map_two_episodes():
    """256x256 (large-map band mode) with 2000 + 2000 agents, random walls and 'random' placement, 200
    steps of each of two episodes in one env: the band buffers' move order on a thinning map and the
    attack-shuffle LCG across the restart (GridWorld.cc:79-89, :437-478, :662-672)."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    ref = _random_scenario(common.REF_LIB, 256, 2000, 2000, 6, 200, 400, episodes=2)
    got = _random_scenario(common.ORACLE_LIB, 256, 2000, 2000, 6, 200, 400, episodes=2)
    assert len(got) == len(ref) and len(ref) > 200
    first_bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if a != b), None)
    assert first_bad is None, "first divergence at step %s" % first_bad
