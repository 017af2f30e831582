"""parse_mac_pdu (protocol.py:349-596): the oracle against the reference's golden calls (CPU), and
the GPU header extraction (tetra_mac_headers) + host state machine against both (GPU)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

G4 = os.path.join(HERE, "golden", "g4_mac.npz")


def golden_calls():
    g = np.load(G4)
    seq = g["seq"]
    calls = []
    for i in range(len(seq)):
        bits = g["bits"][g["bits_off"][i]:g["bits_off"][i + 1]]
        if g["none"][i]:
            want = None
        else:
            want = dict(pdu_type=int(g["ptype"][i]), encrypted=bool(g["enc"][i]),
                        address=None if g["addr"][i] < 0 else int(g["addr"][i]), length=int(g["length"][i]),
                        data=g["data"][g["data_off"][i]:g["data_off"][i + 1]].tobytes(),
                        fill_bits=int(g["fill"][i]), encryption_mode=int(g["mode"][i]),
                        reassembled_data=(g["reasm_data"][g["reasm_off"][i]:g["reasm_off"][i + 1]].tobytes()
                                          if g["reasm"][i] else None))
        state = dict(mcc=None if g["mcc"][i] < 0 else int(g["mcc"][i]),
                     mnc=None if g["mnc"][i] < 0 else int(g["mnc"][i]),
                     cc=None if g["cc"][i] < 0 else int(g["cc"][i]),
                     n_clear=int(g["n_clear"][i]), n_enc=int(g["n_enc"][i]),
                     frag=g["frag"][g["frag_off"][i]:g["frag_off"][i + 1]].tobytes())
        calls.append((int(seq[i]), bits, want, state))
    return calls


def sequences():
    out = {}
    for s, bits, want, state in golden_calls():
        out.setdefault(s, []).append((bits, want, state))
    return [out[k] for k in sorted(out)]


def test_golden_covers_every_branch():
    calls = golden_calls()
    kinds = {w["pdu_type"] for _, _, w, _ in calls if w}
    assert kinds == {0, 1, 2, 3}
    assert any(w is None for _, _, w, _ in calls)
    assert any(w and w["reassembled_data"] and w["pdu_type"] == 2 for _, _, w, _ in calls)
    assert any(st["mcc"] is not None for _, _, _, st in calls)


def test_oracle_matches_reference_golden():
    import mac
    for seq in sequences():
        p = mac.MacParser()
        for bits, want, state in seq:
            got = p.parse(bits)
            assert got == want, (bits.tolist(), got, want)
            assert (p.mcc, p.mnc, p.colour_code, p.n_clear, p.n_enc, bytes(p.fragment_buffer)) == \
                (state["mcc"], state["mnc"], state["cc"], state["n_clear"], state["n_enc"], state["frag"])


def _as_dict(pdu):
    if pdu is None:
        return None
    return dict(pdu_type=pdu.pdu_type.value, encrypted=bool(pdu.encrypted), address=pdu.address, length=pdu.length,
                data=pdu.data, fill_bits=int(pdu.fill_bits), encryption_mode=int(pdu.encryption_mode),
                reassembled_data=pdu.reassembled_data)


@pytest.mark.gpu
def test_gpu_parse_mac_pdu_matches_golden():
    """One call at a time through the drop-in method (a one-frame launch each)."""
    from tetraear.core.protocol import TetraProtocolParser
    for seq in sequences():
        p = TetraProtocolParser()
        for bits, want, state in seq:
            assert _as_dict(p.parse_mac_pdu(bits.astype(np.int64))) == want
            assert (p.mcc, p.mnc, p.colour_code, p.stats["clear_mode_frames"], p.stats["encrypted_frames"],
                    bytes(p.fragment_buffer)) == (state["mcc"], state["mnc"], state["cc"], state["n_clear"],
                                                  state["n_enc"], state["frag"])


@pytest.mark.gpu
def test_gpu_parse_mac_pdu_batch_matches_oracle():
    """Every golden sequence in one launch, then random 0/1 vectors of every length up to 600 (one
    launch of 4096 frames) against the oracle, in order on one parser."""
    import mac
    from tetraear.core.protocol import TetraProtocolParser
    for seq in sequences():
        p = TetraProtocolParser()
        got = p.parse_mac_pdu_batch([b for b, _, _ in seq])
        assert [_as_dict(x) for x in got] == [w for _, w, _ in seq]
    rng = np.random.default_rng(7)
    vecs = []
    for i in range(4096):
        L = int(rng.integers(0, 601))
        v = rng.integers(0, 2, L)
        if L >= 35 and rng.random() < 0.5:   # plausible length indicators
            v[29:35] = [(int(rng.integers(0, (L - 35 + 16) // 8 + 2)) >> (5 - k)) & 1 for k in range(6)]
        vecs.append(v)
    p, o = TetraProtocolParser(), mac.MacParser()
    got = p.parse_mac_pdu_batch(vecs)
    want = [o.parse(v) for v in vecs]
    assert [_as_dict(x) for x in got] == want
    assert (p.mcc, p.mnc, p.colour_code, bytes(p.fragment_buffer)) == (o.mcc, o.mnc, o.colour_code,
                                                                      bytes(o.fragment_buffer))
