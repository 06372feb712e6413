"""Known-answer loudness signals from the standard itself (shared by the CPU and GPU tests).

EBU Tech 3341 ("Loudness Metering: 'EBU Mode' metering to supplement EBU R 128", minimum
requirements test signals) specifies stereo 1 kHz sine sequences and the integrated loudness
a BS.1770-4 meter must report, within +-0.1 LU:

    case 1: 20 s at -23 dBFS                                   -> -23.0 LUFS
    case 2: 20 s at -33 dBFS                                   -> -33.0 LUFS
    case 3: 10 s at -36, 60 s at -23, 10 s at -36 dBFS          -> -23.0 LUFS (relative gate)
    case 4: 10 s -72, 10 s -36, 60 s -23, 10 s -36, 10 s -72   -> -23.0 LUFS (both gates)
    case 5: 20 s at -26, 20.1 s at -20, 20 s at -26 dBFS        -> -23.0 LUFS (energy average)

(dBFS of a sine = its peak relative to full scale.) codes_to_wavs meters ONE channel
(autoencoder.py:172-186 -> pyloudnorm with channel weight 1), and BS.1770's loudness is
-0.691 + 10 log10 of the channel-summed mean square, so the same signal in one channel reads
10 log10 2 = 3.0103 LU lower than the stereo value: these are the expected mono answers."""
import math

import numpy as np

EBU3341 = {
    1: ([(20.0, -23.0)], -23.0),
    2: ([(20.0, -33.0)], -33.0),
    3: ([(10.0, -36.0), (60.0, -23.0), (10.0, -36.0)], -23.0),
    4: ([(10.0, -72.0), (10.0, -36.0), (60.0, -23.0), (10.0, -36.0), (10.0, -72.0)], -23.0),
    5: ([(20.0, -26.0), (20.1, -20.0), (20.0, -26.0)], -23.0),
}
MONO_OFFSET = -10.0 * math.log10(2.0)


def ebu_signal(case: int, rate: int) -> np.ndarray:
    """One channel of EBU Tech 3341 case `case` at `rate` Hz (continuous 1 kHz phase)."""
    segs, _ = EBU3341[case]
    parts, t0 = [], 0
    for dur, dbfs in segs:
        n = int(round(dur * rate))
        t = (np.arange(n) + t0) / rate
        parts.append(10.0 ** (dbfs / 20.0) * np.sin(2.0 * np.pi * 1000.0 * t))
        t0 += n
    return np.concatenate(parts)


def ebu_expected_mono(case: int) -> float:
    return EBU3341[case][1] + MONO_OFFSET
