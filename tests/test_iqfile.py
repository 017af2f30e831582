"""Recorded-IQ file round trips (host) and the SC16 file -> GPU demod path (gpu)."""
import numpy as np
import pytest


def test_sc16_cf32_roundtrip(tmp_path):
    from tetraear.signal import iqfile
    rng = np.random.default_rng(0)
    x = (0.3 * (rng.standard_normal((5000, 3)) + 1j * rng.standard_normal((5000, 3)))).astype(np.complex64)
    iqfile.write_iq(str(tmp_path / "a.sc16"), x)
    iqfile.write_iq(str(tmp_path / "a.cf32"), x)
    m16, f16 = iqfile.open_iq(str(tmp_path / "a.sc16"), channels=3)
    m32, f32 = iqfile.open_iq(str(tmp_path / "a.cf32"), channels=3)
    assert f16 == "sc16" and m16.shape == (5000, 3, 2) and f32 == "cf32" and m32.shape == (5000, 3)
    assert np.array_equal(m32, x)
    q = np.clip(np.round(np.stack([x.real, x.imag], -1) * 32768), -32768, 32767).astype(np.int16)
    assert np.array_equal(m16, q)
    assert np.array_equal(iqfile.to_complex64(m16), (q[..., 0] / 32768 + 1j * (q[..., 1] / 32768)).astype(np.complex64))
    ch = list(iqfile.chunks(str(tmp_path / "a.sc16"), chunk=2048, channels=3))
    assert len(ch) == 2 and ch[0].shape == (3, 2048, 2) and np.array_equal(ch[1][1], q[2048:4096, 1])
    with pytest.raises(ValueError):
        iqfile.fmt_of("x.wav")


@pytest.mark.gpu
def test_sc16_file_demod_matches_cf32(tmp_path):
    from tetraear.signal import iqfile
    from tetraear.signal.etsi import synth, EtsiReceiver
    iq = synth(2, 2 * 131072, seed=4, snr_db=18.0)[0]
    iqfile.write_iq(str(tmp_path / "cap.sc16"), iq.T)          # [N, channels] on disk
    rx = EtsiReceiver()
    for blk in iqfile.chunks(str(tmp_path / "cap.sc16"), channels=2):
        a = rx.demod_batch(blk)                                  # SC16 straight to the device
        b = rx.demod_batch(iqfile.to_complex64(blk))
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
