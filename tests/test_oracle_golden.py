"""Pin the CPU oracle against golden vectors recorded from the reference (CPU only)."""
import numpy as np
import pytest

import compat as O
import mac as M
from conftest import decoded_view, iq_to_c64


def test_g1_process_bit_exact(g1):
    z, meta = g1
    for i, m in enumerate(meta):
        x = iq_to_c64(z[f"c{i}_iq"])
        p = O.SignalProcessor(m["fs"])
        hard = p.process(x, m["freq_offset"])
        assert np.array_equal(hard, z[f"c{i}_hard"]), (i, m)
        assert p.symbols.dtype == z[f"c{i}_symbols"].dtype, (i, m)
        assert np.array_equal(p.symbols, z[f"c{i}_symbols"]), (i, m)


def test_g1_intermediates_bit_exact(g1):
    z, meta = g1
    for i, m in enumerate(meta):
        if m["n"] == 0:
            continue
        x = iq_to_c64(z[f"c{i}_iq"])
        dec = O.decimate(x, m["q"]) if m["dec_ok"] else x
        assert np.array_equal(dec, z[f"c{i}_decimated"]), (i, m)
        if f"c{i}_filtered" in z.files:
            rate = m["fs"] / m["q"] if m["dec_ok"] else m["fs"]
            p = O.SignalProcessor(m["fs"])
            sh = p.frequency_shift(dec, m["freq_offset"], rate) if m["freq_offset"] else dec
            assert np.array_equal(sh, z[f"c{i}_shifted"]), (i, m)
            f = p.filter_signal(sh, 25000, rate)
            assert f.dtype == z[f"c{i}_filtered"].dtype and np.array_equal(f, z[f"c{i}_filtered"]), (i, m)


def test_g1_direct_method_calls(g1):
    z, _ = g1
    p = O.SignalProcessor()
    x = z["direct_x128"]
    assert np.array_equal(p.filter_signal(x, bandwidth=25000), z["direct_filter_25k"])
    assert np.array_equal(p.filter_signal(x, bandwidth=50000), z["direct_filter_50k"])
    assert np.array_equal(p.demodulate_dqpsk(x), z["direct_demod"])
    assert np.array_equal(p.extract_symbols(x), z["direct_extract"])
    assert np.array_equal(p.extract_symbols(x, sample_rate=1.0e6), z["direct_extract_1M"])
    assert np.array_equal(p.frequency_shift(x, 1000), z["direct_shift_1k"])


def test_g2_sync_and_frames(g2):
    z, recs = g2
    for i, r in enumerate(recs):
        sym = z[f"s{i}_sym"]
        bits, mapped = O.symbols_to_bits(sym)
        assert np.array_equal(bits, z[f"s{i}_bits"]) and np.array_equal(mapped, z[f"s{i}_mapped"]), i
        for thr in (0.9, 0.85, 0.8, 0.75, 0.7):
            pos, mc = O.find_sync(bits, threshold=thr, return_max_corr=True)
            assert pos == r[f"fs_{thr}"][0] and mc == r[f"fs_{thr}"][1], (i, thr)
        assert O.decode_syncs(bits) == r["syncs"], i
        frames = O.decode_frames(sym)
        assert len(frames) == len(r["frames"]), i
        for f, g in zip(frames, r["frames"]):
            assert (f["pos"], f["start"], f["number"], f["nbits"]) == (g["pos"], g["start"], g["number"], g["nbits"])
            if g["nbits"] >= 510:
                assert {5: "Synchronization", 2: "NormalDownlink"}[f["burst_type"]] == g["burst_type"]
                assert f["crc_ok"] == g["crc_ok"] and f["header"] == g["header"]
                assert list(f["ts"]) == g["ts"] and list(f["data"]) == g["data"]


def test_g2_decode_mac_stage(g2):
    """decode() through decode_frame's MAC PDU stage (decoder.py:994-1100): the frames the
    reference keeps and their mac_pdu / encrypted / encryption_algorithm, for all streams of g2
    (including the round-3 MAC streams: CRC-good and -bad slots, sync bursts, fragment chains)."""
    z, recs = g2
    kept = dropped = 0
    for i, r in enumerate(recs):
        mp = M.MacParser()
        got = O.decode_with_mac(z[f"s{i}_sym"], mp)
        assert got == [decoded_view(d) for d in r["decoded"]], i
        assert (mp.n_clear, mp.n_enc) == (r["stats"]["clear_mode_frames"], r["stats"]["encrypted_frames"]), i
        kept += len(got)
        dropped += sum(f["nbits"] >= 510 for f in r["frames"]) - len(got)
    assert kept > 100 and dropped > 10


def test_g2_upper_mac_gap_declared(g2):
    """The gap between the build's decode() frames and the reference's is exactly the upper MAC
    (decoder.py:1055-1117; TetraDecoder.upper_mac): every recorded reference frame's keys are the
    ones decoded_view compares plus frame-dict constants, its 'upper_keys' lie in UPPER_MAC_KEYS and
    its additional_info beyond the description / encryption_mode in UPPER_MAC_INFO.  A reference
    field outside these sets would fail here instead of going unnoticed."""
    from conftest import UPPER_MAC_KEYS, UPPER_MAC_INFO
    _, recs = g2
    base = {"number", "timeslot", "type", "header", "position", "burst_crc", "encrypted", "encryption_algorithm",
            "additional_info", "mac_pdu", "upper_keys"}
    seen_upper, seen_info = set(), set()
    for r in recs:
        for d in r["decoded"]:
            assert set(d) <= base, set(d) - base
            seen_upper |= set(d["upper_keys"])
            seen_info |= set(d["additional_info"]) - {"description", "encryption_mode"}
    assert seen_upper <= UPPER_MAC_KEYS and seen_info <= UPPER_MAC_INFO, (seen_upper, seen_info)
    assert seen_upper and seen_info   # the recorded streams do exercise the upper MAC


def test_g3_crc_and_bursts(g3):
    z = g3
    assert int("".join(map(str, z["kat_crc"])), 2) == 0x29B1
    assert int("".join(map(str, O.calculate_crc16(
        np.array([(b >> (7 - k)) & 1 for b in b"123456789" for k in range(8)])))), 2) == 0x29B1
    for v, c, ok in zip(z["crc_vecs"], z["crc_of_vecs"], z["check_crc"]):
        assert np.array_equal(O.calculate_crc16(v), c)
        assert O.check_crc(v) == bool(ok)
    for v, ok in zip(z["crc510_vecs"], z["check510"]):
        assert O.check_crc(v) == bool(ok)
    for n, ok in enumerate(z["crc_short"]):
        assert O.check_crc(np.ones(n, int)) == bool(ok)
    for s, L, t, ts, d, ok in zip(z["burst_syms"], z["burst_len"], z["burst_type"], z["burst_ts"],
                                  z["burst_data"], z["burst_crc_ok"]):
        bt, bts, bd, bok = O.parse_burst_fields(s[:L])
        assert bt == t and bok == bool(ok)
        assert np.array_equal(bts, ts[ts != 255]) and np.array_equal(bd, d[d != 255])
