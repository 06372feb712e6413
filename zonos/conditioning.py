"""`zonos.conditioning` import surface (reference zonos/conditioning.py): make_cond_dict, the
phoneme tokenizer and the PrefixConditioner (one HIP launch, zonos_amd/conditioning.py). The
eSpeak front end is pluggable with set_phonemizer (eSpeak is absent from this image)."""
from zonos_amd.conditioning import (PrefixConditioner, get_symbol_ids, make_cond_dict, phonemize,  # noqa: F401
                                    set_phonemizer, supported_language_codes, tokenize_phonemes)
