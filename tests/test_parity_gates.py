"""The film gates (tests/_parity.py) must fail on films that are wrong in the
ways a GPU film-write, splat or piece bug would make them wrong, and pass the
oracle's own film and a film off by float summation order only.  CPU only:
the damaged films are the oracle's (counter RNG, the streams the GPU draws).

Damage (the writes the gates guard are the splat and the film write of
bidirPathTracing.cpp:110-118, :263):
  * a zeroed 8-row band -- one camera tile row of the film not written;
  * a dropped piece -- one range of path indices of one iteration not
    rendered (its camera pixels and its light paths' splats missing);
  * one film row's splats shifted by one pixel (an orientation / rounding bug
    in the raster position of connectToCamera);
  * one lit pixel off by 1e-3 of its value, and one light path's splat lost
    (the round-5 defect: EPS-black splats dropped, bidirPathTracing.cpp:354).
The -m gpu suite repeats the band, the row shift and the single pixel on the
1080p frame (tests/test_gpu.py::test_bdpt_1080p_matches_oracle_counter_rng).
"""
import numpy as np
import pytest

import _oracle
import _parity
import _scenes

# (case, scene maker, W, H, iterations, seed, control_length, piece)
CASES = [
    ("bdpt_torus256x256_i2_s5", lambda: _scenes.torus(256, 256), 256, 256, 2, 5, 3, (20480, 24576)),
    ("bdpt_cbox64x48_i3_s5489_ctl0", lambda: _scenes.cbox(64, 48, "bdpt"), 64, 48, 3, 5489, 0, (1024, 1536)),
    ("bdpt_torus64x64_i4_s5489", lambda: _scenes.torus(64, 64), 64, 64, 4, 5489, 3, (1024, 1536)),
]
_films = {}


def film(case):
    if case not in _films:
        _, maker, W, H, it, seed, ctl, _ = next(c for c in CASES if c[0] == case)
        o = _oracle.Scene(maker())
        full, _ = o.bdpt(W, H, it, seed, mode=1, control_length=ctl)
        _films[case] = (o, full)
    return _films[case]


def _fails(damaged, ref, case):
    try:
        _parity.assert_film_parity(damaged, ref, case=case)
    except AssertionError:
        return True
    return False


def _energy_rows(f):
    return np.argsort(-np.abs(f).sum(axis=(1, 2)))


@pytest.mark.parametrize("case", [c[0] for c in CASES])
def test_oracle_film_passes_its_own_gates(case):
    _, ref = film(case)
    _parity.assert_film_parity(ref.copy(), ref, case=case)
    # and a film off by float rounding only (the GPU's non-split pixels)
    noisy = (ref.astype(np.float64) * (1 + 1e-7 * np.random.default_rng(1).standard_normal(ref.shape)))
    _parity.assert_film_parity(noisy.astype(np.float32), ref, case=case)


@pytest.mark.parametrize("case", [c[0] for c in CASES])
def test_zeroed_band_fails(case):
    _, ref = film(case)
    H = ref.shape[0]
    # the 8-row tile band holding the most energy, and the one holding the least non-zero energy
    sums = np.abs(ref).reshape(H // 8, 8, -1).sum(axis=(1, 2))
    nonzero = np.nonzero(sums > 0)[0]
    for band in (int(np.argmax(sums)), int(nonzero[np.argmin(sums[nonzero])])):
        dmg = ref.copy()
        dmg[8 * band:8 * band + 8] = 0
        assert _fails(dmg, ref, case), (case, band)


@pytest.mark.parametrize("case", [c[0] for c in CASES])
def test_dropped_piece_fails(case):
    o, ref = film(case)
    _, maker, W, H, it, seed, ctl, (a, b) = next(c for c in CASES if c[0] == case)
    piece, _ = o.bdpt(W, H, 1, seed, mode=1, control_length=ctl, iter_begin=it - 1, path_range=(a, b))
    assert piece.any()
    dmg = (ref.astype(np.float64) - piece).clip(min=0).astype(np.float32)
    assert _fails(dmg, ref, case), case


@pytest.mark.parametrize("case", [c[0] for c in CASES])
def test_splat_row_shifted_by_one_pixel_fails(case):
    _, ref = film(case)
    for row in _energy_rows(ref)[:3]:
        dmg = ref.copy()
        dmg[row] = np.roll(ref[row], 1, axis=0)
        assert _fails(dmg, ref, case), (case, int(row))


def test_single_pixel_errors_fail():
    """Every pixel is gated: one lit pixel 1e-3 too bright fails, in the
    brightest and in a dim lit pixel, and so does a pixel a single light
    path's splat is missing from."""
    case = "bdpt_torus256x256_i2_s5"
    o, ref = film(case)
    lit = np.argwhere(ref.any(axis=-1))
    lum = ref[tuple(lit.T)].sum(-1)
    for y, x in (lit[int(np.argmax(lum))], lit[int(np.argsort(lum)[len(lum) // 10])]):
        dmg = ref.copy()
        dmg[y, x] *= 1.001
        assert _fails(dmg, ref, case), (int(y), int(x))
    # one light path's splat gone: render one path of the last iteration alone
    _, _, W, H, it, seed, ctl, _ = next(c for c in CASES if c[0] == case)
    for p in range(0, W * H, 97):
        one, _ = o.bdpt(W, H, 1, seed, mode=1, control_length=ctl, iter_begin=it - 1, path_range=(p, p + 1))
        one.reshape(-1, 3)[p] = 0  # keep only what the path wrote elsewhere: its splats
        if one.any():
            break
    assert one.any()
    dmg = (ref.astype(np.float64) - one).clip(min=0).astype(np.float32)
    assert _fails(dmg, ref, case)
