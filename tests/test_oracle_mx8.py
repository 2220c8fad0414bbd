"""CPU: pin the MX-fp8 oracle (oracle/mx8.py) — e4m3 encoding against the OCP value table and torch's own
float8_e4m3fn cast, the block-exponent rule on known answers, and the scale-plane layout."""
import numpy as np
import pytest
import torch

from oracle import mx8


def test_e4m3_table_known_values():
    t = mx8.e4m3_value_table()
    assert t[0x38] == 1.0 and t[0x7E] == 448.0 and t[0x01] == 2.0 ** -9 and t[0x08] == 2.0 ** -6
    assert t[0xB8] == -1.0 and t[0x00] == 0.0 and np.isnan(t[0x7F]) and np.isnan(t[0xFF])
    assert t[0x3C] == 1.5 and t[0x30] == 0.5 and t[0x07] == 7 * 2.0 ** -9


def test_e4m3_encode_round_trips_every_finite_code():
    t = mx8.e4m3_value_table()
    codes = np.array([b for b in range(256) if np.isfinite(t[b]) and b != 0x80])   # -0 encodes as +0's sign bit
    assert np.array_equal(mx8.e4m3_encode(t[codes]), codes.astype(np.uint8))


def test_e4m3_encode_matches_torch_cast():
    rng = np.random.default_rng(0)
    t = mx8.e4m3_value_table()
    pos = np.sort(t[np.isfinite(t) & (t >= 0)])
    ties = (pos[:-1] + pos[1:]) / 2                  # exactly half-way between neighbouring codes: to even
    x = np.concatenate([rng.uniform(-448, 448, 20000), rng.normal(0, 1e-2, 20000), rng.normal(0, 1e-3, 5000),
                        ties, -ties, [448.0, -448.0, 0.0]])
    x = x[np.abs(x) <= 448].astype(np.float32)
    ref = torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    got = mx8.e4m3_encode(x)
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:10]


@pytest.mark.parametrize("amax,E", [(1.0, -8), (1.75, -8), (1.7578125, -7), (448.0, 0), (450.0, 1), (3e38, 120),
                                    (0.0, -127), (1e-39, -127)])
def test_block_exponent_known_answers(amax, E):
    bits = (np.array([amax], np.float32).view(np.uint32) >> 16).astype(np.int64) & 0x7FFF
    assert int(mx8.block_exponent(bits)[0]) == E
    if amax > 0:   # no element saturates, and the top of the block uses the top binade
        assert amax * 2.0 ** -E <= 448.0


def test_quantize_dequantize_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.normal(size=(37, 256)) * np.exp2(rng.integers(-30, 30, (37, 1)))).astype(np.float32)
    bits = (x.view(np.uint32) >> 16).astype(np.uint16)              # truncate to bf16 (any bf16 will do)
    xb = (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    codes, sc = mx8.quantize(bits)
    d = mx8.dequantize(codes, sc)
    ulp_floor = np.repeat(np.exp2(sc - 127.0 - 9), 32, axis=1)      # subnormal step of the block
    assert np.all(np.abs(d - xb) <= np.abs(xb) * 2.0 ** -4 + ulp_floor)


def test_scale_planes_layout():
    rows, K, lds = 130, 256, 192
    sb = np.arange(rows * (K // 32)).reshape(rows, K // 32) % 251
    planes = mx8.pack_scales(sb, lds).view(np.uint8).reshape(-1)
    for r in (0, 15, 16, 63, 64, 129):
        for kb in range(K // 32):
            assert planes[mx8.scale_byte_index(r, kb * 32, lds)] == sb[r, kb]
    # a GEMM lane (brick row r16, K-block fq) finds its 4 fragments' scales in one word
    w = planes.view(np.uint32)
    r16, fq = 5, 2
    word = int(w[0 * lds + 64 + fq * 16 + r16])     # brick 1 (rows 64..127), plane 0
    assert [(word >> (8 * f)) & 0xFF for f in range(4)] == [sb[64 + 16 * f + r16, fq] for f in range(4)]
