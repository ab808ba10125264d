"""CPU oracle for the GRPO/PPO hot path — TEST INFRASTRUCTURE ONLY.

This package is a line-cited CPU restatement of the reference's algorithms
(shiwanghua/swh-trl, a TRL 0.21.0.dev0 fork).  Citations are `path:line`
relative to the reference tree.

Rules:
  * Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline`
    leg may import anything from here, and only as the checker / the timed
    CPU baseline.  The product (`swh_trl_amd`) never imports it and has no
    CPU fallback.
  * The reference itself may not be imported or run (SURVEY.md §8c records
    the denial).  The restatement is pinned by the known-answer tests the
    reference's own test-suite holds, transcribed as data into
    `tests/golden/reference_kats.json`, and by third-party oracles that the
    survey allows (installed torch / transformers) for third-party ops.
  * Functions that no reference test pins are marked "parity unpinned" in
    their docstring.
"""
