"""Load the reference's Python modules from /root/reference for golden-vector generation.

TEST INFRASTRUCTURE ONLY, and only in the build container: /root/reference does not exist on
the GPU box and nothing under tests/ that runs there imports this file.

The reference is a partial AutoAWQ fork whose files sit at the top level but import each other
as ``awq.*``.  Several of those imports name modules that are absent from the
snapshot (``awq.modules.*``, ``awq.quantize.genCodeBook``'s kmeans dependency,
``hadamard_transform``, ``torchsummary``, ``diffusers``).  We register light stubs for exactly
those names so that the reference's own source files execute unchanged from their read-only
location; nothing is copied.  The stubs only satisfy ``import`` statements: none of them is
reached by the functions whose outputs become golden vectors (codebook quantization is off,
the calibration data path is not called).
"""
import importlib.util
import sys
import types

REF = "/root/reference"


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__path__ = []  # allow sub-imports
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class _Unreachable:
    def __init__(self, *a, **k):
        raise RuntimeError("stubbed reference dependency reached during golden generation")


def load_reference():
    """Return a namespace with the reference modules used for golden generation."""
    if "awq.quantize.fake_quant" in sys.modules:
        m = sys.modules
        return types.SimpleNamespace(fake_quant=m["awq.quantize.fake_quant"],
                                     quantizer=m["awq.quantize.quantizer"],
                                     quantizer_SQ=m["awq.quantize.quantizer_SQ"],
                                     calib_data=m["awq.utils.calib_data"])
    for pkg in ("awq", "awq.quantize", "awq.utils", "awq.modules", "awq.models"):
        _stub(pkg)
    # absent third-party / absent-in-snapshot modules (import-only stubs)
    _stub("hadamard_transform", hadamard_transform=_Unreachable)
    _stub("awq.quantize.genCodeBook", codeBookQuant=_Unreachable)
    _stub("torchsummary", summary=_Unreachable)
    _stub("awq.modules.linear", WQLinear_GEMM=_Unreachable, WQLinear_GEMV=_Unreachable,
          WQLinear_Marlin=_Unreachable, WQLinear_GEMVFast=_Unreachable)
    _stub("awq.modules.act", ScaledActivation=_Unreachable)
    # diffusers is absent: calib_data.py needs PipelineCallback, DiffusionPipeline,
    # diffusers.utils.torch_utils.randn_tensor at import/annotation time only.
    class _PipelineCallback:
        def __init__(self, *a, **k):
            pass
    d = _stub("diffusers", DiffusionPipeline=object)
    _stub("diffusers.callbacks", PipelineCallback=_PipelineCallback)
    d.callbacks = sys.modules["diffusers.callbacks"]
    _stub("diffusers.utils")
    _stub("diffusers.utils.torch_utils", randn_tensor=_Unreachable)
    d.utils = sys.modules["diffusers.utils"]
    d.utils.torch_utils = sys.modules["diffusers.utils.torch_utils"]
    _stub("awq.models.base", diffusers=d)

    _load("awq.utils.utils", f"{REF}/utils/utils.py")
    _load("awq.utils.module", f"{REF}/utils/module.py")
    fq = _load("awq.quantize.fake_quant", f"{REF}/quantize/fake_quant.py")
    cd = _load("awq.utils.calib_data", f"{REF}/utils/calib_data.py")
    _load("awq.quantize.scale", f"{REF}/quantize/scale.py")
    qz = _load("awq.quantize.quantizer", f"{REF}/quantize/quantizer.py")
    sq = _load("awq.quantize.quantizer_SQ", f"{REF}/quantize/quantizer_SQ.py")
    return types.SimpleNamespace(fake_quant=fq, quantizer=qz, quantizer_SQ=sq, calib_data=cd)


def load_sd15_adapter():
    """models/StableDiffusion1_x.py (its mean_of_dict uses no instance state).  Its imports are
    torch / BaseAWQForDiffusion / QUANTISABLE_COMPONENTS from .base (the base module needs the
    absent diffusers and AutoAWQ runtime: import-only stand-ins here) and diffusers'
    BasicTransformerBlock (absent: an import-only stand-in)."""
    import torch
    load_reference()
    base = sys.modules["awq.models.base"]
    base.torch = torch
    base.BaseAWQForDiffusion = type("BaseAWQForDiffusion", (), {})
    base.QUANTISABLE_COMPONENTS = {}
    d = sys.modules["diffusers"]
    _stub("diffusers.models")
    _stub("diffusers.models.attention", BasicTransformerBlock=_Unreachable)
    d.models = sys.modules["diffusers.models"]
    d.models.attention = sys.modules["diffusers.models.attention"]
    return _load("awq.models.StableDiffusion1_x", f"{REF}/models/StableDiffusion1_x.py")
