"""`zonos.model` import surface (reference zonos/model.py) served by the MI355X engine.

Callers written against the reference -- sample.py:9-11, zonos_batch_cli.py:13-15 -- import
``from zonos.model import Zonos`` and run unchanged; the model is zonos_amd.model.Zonos
(generate() on the HIP engine, hipGraph-captured decode step). This directory is a namespace
package like the reference's (no __init__.py)."""
from zonos_amd.model import Zonos  # noqa: F401

from .backbone import BACKBONES

DEFAULT_BACKBONE_CLS = next(iter(BACKBONES.values()))     # model.py:19
