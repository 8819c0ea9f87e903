"""The oracle reproduces the committed golden fixtures bit for bit (tests/golden/make_golden.py)."""
import pytest

import golden_util as G
import oracle


@pytest.mark.parametrize("name", G.names())
def test_oracle_matches_golden(name):
    scene, org, params, fresh, expected, counts = G.load(name)
    got = oracle.run(scene, params, org, fresh, threads=4)[1]
    eq = fresh.equal(expected)
    assert all(eq.values()), eq
    assert got == counts


def test_fixtures_present():
    assert len(G.names()) >= 6
