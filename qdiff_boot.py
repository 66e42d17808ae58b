"""Register the in-tree package directory ``quantization---diffusion-models_amd/`` as ``qdiff``.

The directory name required by the project layout is not a Python identifier, so it cannot be
imported by name.  ``import qdiff_boot`` (done by ``AWQ.py``, ``bench.py``, ``__graft_entry__``
and ``tests/conftest.py``) loads it under the importable name ``qdiff``; afterwards
``import qdiff`` / ``from qdiff.unet import ...`` work normally.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "quantization---diffusion-models_amd")


def load():
    if "qdiff" in sys.modules:
        return sys.modules["qdiff"]
    spec = importlib.util.spec_from_file_location(
        "qdiff", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["qdiff"] = mod
    spec.loader.exec_module(mod)
    return mod


qdiff = load()
