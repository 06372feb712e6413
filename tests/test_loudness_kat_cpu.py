"""CPU: the loudness restatement (oracle/loudness_ref.py, pyloudnorm 0.1.1's algorithm) against
the standard's own known answers -- EBU Tech 3341 cases 1-5 (tests/loudness_kat.py), at the
DAC's 44.1 kHz and at the standard's 48 kHz, within the +-0.1 LU the standard allows. pyloudnorm
itself is not installed; this pins the meter to BS.1770-4 / EBU R 128 instead."""
import pytest

from oracle import loudness_ref

from .loudness_kat import EBU3341, ebu_expected_mono, ebu_signal


@pytest.mark.parametrize("rate", [44100, 48000])
@pytest.mark.parametrize("case", sorted(EBU3341))
def test_ebu3341_integrated_loudness(case, rate):
    got = loudness_ref.integrated_loudness(ebu_signal(case, rate), rate, 0.400)
    assert abs(got - ebu_expected_mono(case)) <= 0.1, (case, rate, got, ebu_expected_mono(case))
