"""exacto_amd — MI355X (gfx950) ciphertext-multiplication path of exacto behind a C ABI.

The compute lives in ``lib/libexacto_hip.so`` (hand-written HIP kernels, see
``csrc/``); ``_ffi`` binds its C ABI (include/exacto_hip.h).  ``bfv`` / ``dbfv`` /
``params`` mirror the reference's Rust API surface (exacto::bfv::eval,
exacto::dbfv::eval, exacto::params) on batched device-resident ciphertexts.
"""

__version__ = "0.1.0"
