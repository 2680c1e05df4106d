"""CPU oracle for the exacto ciphertext-multiplication hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``, and
only as the checker.  The product path (``exacto_amd`` + ``libexacto_hip.so``)
never imports, links or calls this package.

What it is
----------
An exact-integer restatement (Python ints, so u128/i128/BigInt semantics are
reproduced without overflow) of the reference Rust crate RajeshRk18/exacto on
the path ``bfv_mul_and_relin`` / ``relinearize`` / ``dbfv_mul``.  Every
function cites the reference ``path:line`` it restates.

Pinning status
--------------------------------------
* The reference is Rust; no cargo/rustc exists in this image and the NTT lives
  in the un-vendored crate ``concrete-ntt 0.2.0`` (Cargo.lock:142-149), so the
  reference cannot be built or run here.  The oracle is pinned by the
  reference's own known-answer tests (tests/golden/kats.json, every KAT cites
  its source line) and by its decrypt-level functional tests.
* Coefficient-domain results are pinned.  The NTT *evaluation order / root*
  of concrete-ntt is not observable from the reference's tests
  ("NTT-domain parity unpinned"); this build documents its own convention
  (``ring.NttPlan``) and every parity claim on NTT-domain data is made after
  the inverse transform.
* Q >= 2^64 with L >= 2 limbs: the reference's ``RnsPoly::to_coeff_poly``
  overflows (src/ring/rns.rs:135,147,150), so ``relinearize`` has no defined
  output there.  The oracle uses the "extension semantics" of SURVEY.md §8(c):
  exact CRT, same balanced-digit rule; it coincides with the reference for
  every L = 1 config and for multi-limb Q < 2^64.
"""

from . import modular, ring, params, bfv, dbfv  # noqa: F401
