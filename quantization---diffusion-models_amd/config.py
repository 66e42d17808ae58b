"""AwqConfig: the quantization config dataclass of models/_config.py:8-119 (same keys/defaults).

Defaults (_config.py:10-23): w_bit=4, a_bit=16, q_group_size=128, zero_point=True (unused by the
fake-quant modules), version='fake_act', weight_quant_type='group',
weight_quant_conv_type='per_channel', act_quant_conv_type='per_channel',
act_quant_conv_group_size=1, quantize_act=False.
"""
import json
import os
from dataclasses import dataclass, field, fields
from typing import Dict, List, Optional


@dataclass
class AwqConfig:
    quant_method: str = field(default="awq")
    zero_point: bool = field(default=True)
    q_group_size: int = field(default=128)
    w_bit: int = field(default=4)
    wv_bit: int = field(default=4)
    a_bit: int = field(default=16)
    version: str = field(default="fake_act")
    modules_to_not_convert: Optional[List] = None
    weight_quant_conv_type: str = field(default="per_channel")
    weight_quant_type: str = field(default="group")
    act_quant_conv_type: str = field(default="per_channel")
    act_quant_conv_group_size: int = field(default=1)
    quantize_act: bool = field(default=False)

    config_file_name = "config.json"

    @classmethod
    def from_dict(cls, quant_config: Dict = {}):
        """_config.py:25-33 (unknown keys raise TypeError, as dataclass construction does)."""
        if not quant_config:
            return cls()
        cfg = cls(**quant_config)
        cfg.version = cfg.version.lower()
        return cfg

    @classmethod
    def from_pretrained(cls, save_dir: str, is_diffusion_model=False, **kwargs):
        """_config.py:35-84.  Diffusion models get defaults (:81-82).  For non-diffusion
        directories the local config.json's ``quantization_config`` is read (no hub access)."""
        if is_diffusion_model:
            return cls()
        path = os.path.join(save_dir, cls.config_file_name)
        if os.path.exists(path):
            with open(path, "r", encoding="utf-8") as f:
                qc = json.load(f).get("quantization_config")
            if qc is not None:
                return cls(**cls.from_transformers_dict(cls, qc))
        return cls()

    def to_dict(self):
        return {"zero_point": self.zero_point, "q_group_size": self.q_group_size, "w_bit": self.w_bit,
                "wv_bit": self.wv_bit, "a_bit": self.a_bit, "version": self.version,
                "modules_to_not_convert": self.modules_to_not_convert}

    def to_transformers_dict(self):
        """_config.py:97-107 (the dict injected into each quantized component's config.json)."""
        return {"quant_method": self.quant_method, "zero_point": self.zero_point,
                "group_size": self.q_group_size, "bits": self.w_bit, "vbits": self.wv_bit,
                "act_bits": self.a_bit, "version": self.version.lower(),
                "modules_to_not_convert": self.modules_to_not_convert}

    def from_transformers_dict(self, transformers_dict: Dict):
        """_config.py:109-119 (called unbound in the reference: ``cls.from_transformers_dict(cls, d)``)."""
        d = transformers_dict
        return {"quant_method": d.get("quant_method"), "zero_point": d.get("zero_point"),
                "q_group_size": d.get("group_size"), "w_bit": d.get("bits"), "wv_bit": d.get("vbits"),
                "a_bit": d.get("act_bits"), "version": d.get("version"),
                "modules_to_not_convert": d.get("modules_to_not_convert")}

    def full_dict(self):
        """All fields (our own on-disk format keeps the conv/act granularity keys too)."""
        return {f.name: getattr(self, f.name) for f in fields(self)}
