"""GPU: the SAT edge query on sign bits (narrowphase.hip groupEdgeQueryBits,
box pairs) against the oracle's products (reference
src/physics/narrowphase.cpp:474-540, queryEdgeDirections / isMinkowskiFace).

The sign rule is exact for table entries that are exactly zero (the product
is zero, the test fails) or at least 2^-62 in magnitude; axis-aligned boxes
make many entries exactly zero, rotated piles make none.  Both kinds of world
run bit-exact against the oracle every step: candidates and contacts."""
import numpy as np
import pytest

from oracle_lib import gen_collisions_inits
from test_lds_fallback_gpu import _lockstep, _pair

pytestmark = pytest.mark.gpu


def _aligned_rows(W, n, spacing, z0=0.95, layers=2):
    """Identity-rotated cubes in overlapping rows and layers: the face
    queries do not separate them, so the edge query runs on tables full of
    exact zeros."""
    pos = np.zeros((W, n, 3), np.float32)
    rot = np.zeros((W, n, 4), np.float32)
    rot[..., 0] = 1.0
    per_layer = (n + layers - 1) // layers
    side = int(np.ceil(np.sqrt(per_layer)))
    for w in range(W):
        i = np.arange(n)
        layer, k = i // per_layer, i % per_layer
        pos[w, :, 0] = (k % side) * spacing + 0.01 * w
        pos[w, :, 1] = (k // side) * spacing
        pos[w, :, 2] = z0 + layer * spacing
    return pos, rot


def test_axis_aligned_boxes_bit_exact():
    W, n = 4, 32
    pos, rot = _aligned_rows(W, n, spacing=1.9)
    sim, orc = _pair(W, n, pos, rot)
    _lockstep(sim, orc, W, 40)
    _, k = sim.counts()
    assert np.all(k > 0), k


def test_rotated_piles_bit_exact():
    W, n = 8, 64
    pos, rot = gen_collisions_inits(W, n, seed=23)
    sim, orc = _pair(W, n, pos, rot)
    _lockstep(sim, orc, W, 80)
