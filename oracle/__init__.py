"""TEST INFRASTRUCTURE — CPU oracle for the ZeRO sharded-optimizer step.

This package is the *checker*, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The shipped path (``zero_amd``) never imports,
links or calls anything here, and fails loudly if its HIP library is missing.

Contents
  zero_oracle.py  numpy restatement of the reference ShardedOptimizer semantics (ownership,
                  ZeRO-1 carry, ZeRO-2 data-parallel Adam, ZeRO-3 reduce-and-discard) and of the
                  torch.optim.Adam update it delegates to, each function citing the reference
                  file:line it follows.
  adam_oracle.c   plain-C restatement of the same Adam update (fp32 and bf16-grad/bf16-param with
                  fp32 master), used for bit-level checks and as the timed CPU baseline.

Pinning: the restatement is checked against golden vectors produced by running the reference's
own ShardedOptimizer (gloo/CPU) and torch.optim.Adam in the build container
(tests/golden/make_golden.py → tests/golden/*.npz; tests/test_oracle.py).  The bf16 mixed-precision
mode has no reference counterpart (the reference is fp32-only): its fp32 arithmetic is pinned by the
same fixtures, the bf16 rounding of grads/params is parity-unpinned beyond that.
"""
