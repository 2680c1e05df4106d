"""exacto_amd — MI355X (gfx950) ciphertext-multiplication path of exacto behind a C ABI.

The compute lives in ``lib/libexacto_hip.so`` (hand-written HIP kernels, ``csrc/``).
``_ffi`` binds its C ABI (include/exacto_hip.h): ``HipContext`` carries the reference's
operations (exacto::bfv::eval, exacto::bfv::keyswitch, exacto::dbfv::eval, keygen / encrypt /
decrypt, the Galois and bootstrap helpers) on batched host or device-resident ciphertexts.
``dist`` is the multi-GPU layer (batch shards, the output-limb split of one dbfv_mul, RCCL key
broadcast) and ``bootstrap`` the host-side composition of bfv_host.rs.  The C++ mirror of the
Rust API is include/exacto.hpp.
"""

__version__ = "0.4.0"
