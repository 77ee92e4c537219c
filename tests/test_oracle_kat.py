"""Pins the CPU oracle to the reference's own unit tests (CPU only).

oracle/kat.cpp + oracle/kat_sfu.inc transcribe the known-answer vectors of
rangemap_test.go, wraparound_test.go, rtpmunger_test.go, codecmunger/vp8_test.go,
buffer/helpers_test.go, forwarder_test.go (GetTranslationParams*, padding,
blank frames, layers, mute), sequencer_test.go, audio/audiolevel_test.go and
buffer/rtpstats_receiver_test.go, and (oracle/kat_dd.inc) the dependency-descriptor
captures of dependencydescriptor/dependencydescriptorextension_test.go plus
videolayerselector/framenumberwrapper_test.go.  Each KAT runs as its own test case.
"""
import os
import subprocess

import pytest

from tests import oracle_lib


def _kat_names():
    if not os.path.exists(oracle_lib.KAT):
        oracle_lib.build()
    out = subprocess.run([oracle_lib.KAT, "--list"], check=True, capture_output=True, text=True).stdout
    return [x for x in out.split() if x]


NAMES = _kat_names()


def test_kat_inventory():
    """Every reference test file named in SURVEY.md §8(c) that the oracle covers has KATs."""
    prefixes = ["rangemap", "wraparound", "rtpmunger", "vp8_", "forwarder_", "sequencer", "audiolevel", "ddsel_",
                "rtpstats_receiver", "dd_"]
    for p in prefixes:
        assert any(n.startswith(p) for n in NAMES), p
    assert len(NAMES) >= 40


@pytest.mark.parametrize("name", NAMES)
def test_kat(name):
    r = subprocess.run([oracle_lib.KAT, name], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert ("PASS " + name) in r.stdout
