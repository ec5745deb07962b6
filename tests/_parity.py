"""Film parity gates: the GPU film against the oracle's film drawn from the
same counter-RNG streams (test infrastructure).

Where the two differ, and why (scripts/parity_stats.py measures it;
profiles/r3/parity_stats.jsonl holds the run these gates are set from):
  * OCML and glibc round cosf / sinf / powf differently in the last ulp now and
    then (glibc's cosf itself differs from the correctly rounded value on 1.3 %
    of the sampler's 2^24 inputs).  A BDPT / PT path whose direction moves by
    an ulp almost always lands on the same triangle and adds the same value to
    1e-7; rarely it hits something else ("path split") and one pixel (a splat:
    anywhere) differs completely.  The reference's absolute EPS makes splits
    likelier than the ulp suggests: at torus.scene's scale (coordinates ~1e3,
    an ulp ~6e-5) an ulp-level shift of a hit point decides whether the next
    ray, started EPS along its direction, re-hits its own triangle
    (scripts/debug_path.py traced one such path on both sides: the GPU's second
    light ray re-hit its first triangle at t = 0.007, the oracle's did not).
    Measured: 0-178 split pixels per film (1080p: 8.5e-5 of the frame; the
    64x48 Cornell box, all edges and corners: 17 = 0.55 %), every other pixel
    within 1e-5 relative (PT: the order of the per-sample float atomics,
    <= 1.4e-5).
  * VCM merges light vertices within a radius: an ulp of position flips a
    vertex across the radius somewhere in every few hundred queries, so 3-46 %
    of VCM pixels differ by 1e-4..1e-1 relative.

So a BDPT / PT film passes when
  * at most max(16, 1 % of the) pixels differ by more than `bad_rel` (1e-4)
    relative (the path splits), and
  * on all other pixels the relative RMSE is below `trimmed` (2e-6) and the
    summed difference is below `bias` (2e-7) of the summed film -- ten times
    the largest values measured (2.8e-7 and 1.6e-8 over 13 films).
A 1e-3 change of an MIS weight moves every pixel that weight touches by about
1e-3 x its share of the pixel, and the summed film by 1e-3 x the weighted
strategy's share of the image: above 2e-7 for any strategy worth 0.02 % of
the image (scripts/perturbation_check.sh builds such a library and shows
it).  VCM films pass on whole-film relative RMSE, total bias, the fraction of
flipped-merge pixels and the agreement of the rest, plus the merge counts.
"""
import numpy as np


def film_stats(film, ref, bad_rel=1e-4):
    a = np.asarray(film, np.float64)
    b = np.asarray(ref, np.float64)
    d = a - b
    rms = float(np.sqrt((b ** 2).mean()))
    floor = 1e-3 * float(np.abs(b).mean()) + 1e-30
    rel = np.abs(d) / np.maximum(np.abs(b), floor)
    bad = (rel > bad_rel).any(axis=-1)
    good = ~bad
    dg, bg = d[good], b[good]
    g_rms = float(np.sqrt((bg ** 2).mean())) if bg.size else 0.0
    return {
        "rel_rmse": float(np.sqrt((d ** 2).mean())) / rms if rms > 0 else float("inf"),
        "bias": float(d.sum() / max(np.abs(b).sum(), 1e-30)),
        "bad_pixels": int(bad.sum()),
        "pixels": int(bad.size),
        "trimmed_rel_rmse": float(np.sqrt((dg ** 2).mean())) / g_rms if g_rms > 0 else 0.0,
        "trimmed_bias": float(dg.sum() / max(np.abs(bg).sum(), 1e-30)),
        "rms": rms,
        "ch_rmse": np.sqrt((d ** 2).reshape(-1, d.shape[-1]).mean(axis=0)),
    }


def assert_film_parity(film, ref, *, bad_rel=1e-4, max_bad_frac=1e-2, min_bad=16, trimmed=2e-6, bias=2e-7):
    """BDPT / PT film vs the oracle's (see the module docstring)."""
    s = film_stats(film, ref, bad_rel)
    assert np.all(np.isfinite(film)) and np.asarray(film).min() >= 0, "film not finite / negative"
    if s["rms"] == 0:  # e.g. a 1x1 film that sees no light: black on both sides
        assert not np.asarray(film).any(), "oracle film is black, GPU film is not"
        return s
    assert s["bad_pixels"] <= max(min_bad, max_bad_frac * s["pixels"]), s
    assert s["trimmed_rel_rmse"] < trimmed, s
    assert abs(s["trimmed_bias"]) < bias, s
    # north_star: per-channel RMSE < 1e-3 -- implied by the above, kept explicit
    assert np.all(s["ch_rmse"] < 1e-3), s
    return s


def assert_vcm_parity(film, ref, *, rel_rmse=1e-2, bias=3e-3, max_bad_frac=0.6, trimmed=1e-4):
    """VCM film vs the oracle's: merges flip at the radius (module docstring),
    so up to max_bad_frac of the pixels may differ by > 1e-4; the rest agree
    to `trimmed`, and the whole film to `rel_rmse` and `bias`."""
    s = film_stats(film, ref)
    assert np.all(np.isfinite(film)) and np.asarray(film).min() >= 0, "film not finite / negative"
    assert s["rms"] > 0, "oracle film is black"
    assert s["rel_rmse"] < rel_rmse, s
    assert abs(s["bias"]) < bias, s
    assert s["bad_pixels"] <= max_bad_frac * s["pixels"] + 8, s
    assert s["trimmed_rel_rmse"] < trimmed, s
    assert np.all(s["ch_rmse"] < 1e-3), s
    return s


def assert_ray_counts(st, rst, slack=16, rel=2e-6):
    """Closest / shadow traversal counts: equal up to the rays of split paths
    (measured: at most 9 per film)."""
    for k in ("closest_rays", "shadow_rays"):
        a, b = getattr(st, k), getattr(rst, k)
        assert abs(a - b) <= slack + rel * b, (k, a, b)
