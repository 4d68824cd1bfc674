"""honk_amd -- MI355X (gfx950) native forward path of Honk's keyword-spotting CNNs.

Drop-in for /root/reference/utils/model.py (registry + modules) with the
evaluate()/train() and label() callers; compute on hand-written HIP kernels in
libhonk_hip.so.
"""
from .model import (ConfigType, SerializableModule, SpeechModel, SpeechResModel, find_config, find_model,  # noqa
                    truncated_normal, _configs)

__all__ = ["ConfigType", "SerializableModule", "SpeechModel", "SpeechResModel", "find_config", "find_model",
           "truncated_normal"]
