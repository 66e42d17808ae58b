"""CPU oracle for the quantized-diffusion hot path.

TEST INFRASTRUCTURE, NOT PRODUCT.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``, and only as the
checker (or the timed CPU baseline), never as something the product path calls.

Contents
--------
``fake_quant_np``   numpy restatement of ``quantize/fake_quant.py`` (Appendix A numerics),
                    pinned bit-exactly by ``tests/golden/fake_quant_golden.npz``.
``fake_quant_torch`` the same math on torch-CPU fp16 tensors (what the reference itself runs),
                    pinned by the same fixtures; used inside the CPU UNet.
``modules``         ``OracleWxAxLinear`` / ``OracleWxAxConv2d`` (forward semantics of
                    ``fake_quant.py:170-398``), the diffusion-branch traversal/swap of
                    ``quantizer.py:386-425,491-533`` and ``smooth_ln_fcs``
                    (``quantizer_SQ.py:395-431``).
``unet_ref``        torch-CPU NCHW restatement of the diffusers SD1.5/SDXL UNet (third-party,
                    absent here: parity of the architecture itself is UNPINNED)
                    with fake-quant modules installed; the CPU baseline of bench.py.
``sched_ref``       DDIM scheduler restatement (diffusers, absent: unpinned).
"""
