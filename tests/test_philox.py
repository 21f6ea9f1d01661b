"""Pin the hand-written Philox4x32-10 (oracle C + Python) against rocRAND's
engine output (tests/golden/philox_rocrand.json, made by
tests/golden/gen_philox_rocrand.cpp) — which also matches the Random123
known-answer vectors."""
import json
import pathlib

from oracle import philox as pp

GOLD = json.loads((pathlib.Path(__file__).parent / "golden" / "philox_rocrand.json").read_text())

R123_KAT = [  # Random123 kat_vectors, philox4x32 R=10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_python_philox_vs_rocrand():
    for g in GOLD:
        assert list(pp.philox4x32_10(g["ctr"], g["key"])) == g["out"]


def test_python_philox_random123_kat():
    for ctr, key, out in R123_KAT:
        assert pp.philox4x32_10(ctr, key) == out


def test_c_oracle_philox_vs_rocrand(oracle_mod):
    for g in GOLD:
        assert list(oracle_mod.philox(g["ctr"], g["key"])) == g["out"]


def test_peer_draw_range():
    n = 4096
    for i in (0, 1, 2047, 4095):
        for t in range(8):
            p = pp.peer(0x5EED0002, i, 3, t, n)
            assert 0 <= p < n and p != i
