"""MI355X-native sequential SIFT feature-matching stage (drop-in for the
SequentialMatchingCPU Scanner op of garyjyzhang/scanner-colmap).

Public surface:
  * ``Context`` / ``MatchingOptions`` — the C ABI (include/scm.h) over ctypes;
  * ``scanner_op/`` — the Scanner op/kernel shim over the C ABI (C++);
  * ``feature_matching`` — the job-script mirror of feature_matching.py;
  * ``codecs`` — the io.cc element formats;
  * ``synthetic`` — deterministic synthetic `extraction` tables.
"""
from ._abi import (Context, MatchingOptions, ScmError, default_options,  # noqa: F401
                   load_library, pair_seed, parse_args)

__all__ = ["Context", "MatchingOptions", "ScmError", "default_options", "load_library",
           "pair_seed", "parse_args"]
