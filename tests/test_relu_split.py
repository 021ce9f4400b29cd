"""The ReLU folded into the split-f16 layer-2 operand (csrc layer2_split_relu), emulated on the
host: hi = f16(z) rounded toward zero (v_cvt_pkrtz_f16_f32), lo = f16(clamp(z - hi, 0, 1))
(v_fma_mix_f32 with the clamp bit, then v_cvt_pk_f16_f32), hi' = max(hi, 0) (v_pk_max_f16).
For every z < 2048 (the host's layer-1 bound for relu nodes) hi' + lo is relu(z) to the split's
precision, and exactly 0 for z <= 0."""
import numpy as np


def _f16_rtz(z: np.ndarray) -> np.ndarray:
    h = z.astype(np.float16)                                   # round to nearest even
    over = np.abs(h.astype(np.float64)) > np.abs(z.astype(np.float64))
    h[over] = np.nextafter(h[over], np.float16(0))             # one step toward zero
    return h


def test_folded_relu_split_is_relu():
    rng = np.random.default_rng(0)
    z = np.concatenate([rng.normal(size=20000) * 10.0 ** rng.integers(-6, 3, 20000),
                        rng.uniform(-2047.9, 2047.9, 20000), [0.0, -0.0, 1e-30, -1e-30, 2047.9, -5000.0]])
    z = z.astype(np.float32)
    hi = _f16_rtz(z)
    r = (z.astype(np.float32) - hi.astype(np.float32)).astype(np.float32)   # exact (Sterbenz)
    assert (r[z >= 0] >= 0).all() and (r[z >= 0] < 1).all() and (r[z < 0] <= 0).all()
    lo = np.clip(r, 0.0, 1.0).astype(np.float16)
    hp = np.maximum(hi, np.float16(0))
    got = hp.astype(np.float64) + lo.astype(np.float64)
    want = np.maximum(z.astype(np.float64), 0.0)
    assert (got[z <= 0] == 0).all()
    pos = z > 0
    # relative 2^-21 (hi loses one bit to RTZ, lo carries it); absolute 2^-24: f16 subnormals, as
    # the round-to-nearest split (values below 2^-24 flush to 0 in either)
    assert (np.abs(got[pos] - want[pos]) <= 2.0 ** -21 * want[pos] + 2.0 ** -24).all()
