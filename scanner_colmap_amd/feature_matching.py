"""Command-line mirror of the reference job script `integration/feature_matching.py`
for the GPU op, without Scanner: the `extraction` table comes from a COLMAP
database (or any io.cc element source), the stencil `range(0, overlap)`
(`feature_matching.py:43`) runs on the GPU over the whole table held in HBM,
and the `matching` rows go to a COLMAP database's two_view_geometries table
the way the downstream mapper loads them.

    python -m scanner_colmap_amd.feature_matching --database in.db \
        --output_database out.db --overlap 10

Arguments mirror the reference's (`--overlap`, `--packet_size`); Scanner-only
ones (`--scanner_config`, `--input_table`, `--output_table`) are accepted and
ignored.  `--packet_size` only matters to Scanner's scheduling; the GPU path
batches by pairs instead (SCM_BATCH_PAIRS).
"""
from __future__ import annotations

import argparse
import struct
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--database", required=True, help="COLMAP database with images/keypoints/descriptors")
    ap.add_argument("--output_database", default=None,
                    help="where to write two_view_geometries (default: --database)")
    ap.add_argument("--overlap", type=int, default=10, help="the matching window size")
    ap.add_argument("--packet_size", type=int, default=25, help="accepted for compatibility")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--scanner_config", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--input_table", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--output_table", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args(argv)

    from . import Context
    from .colmap_db import read_extraction, write_two_view_geometries

    ids, kps, descs = read_extraction(a.database)
    if not ids:
        print("no images in the database", file=sys.stderr)
        return 1
    t0 = time.perf_counter()
    ctx = Context(a.device)
    try:
        ctx.table_load(ids, kps, descs)
        pair_rows, tvg_rows = ctx.table_run(a.overlap, 0, len(ids))
    finally:
        ctx.close()
    dt = time.perf_counter() - t0
    pivots = [struct.unpack_from("<Q", b)[0] & 0xFFFFFFFF for b in ids]
    n = write_two_view_geometries(a.output_database or a.database, pivots, pair_rows, tvg_rows)
    print(f"matched {n} image pairs of {len(ids)} images in {dt:.2f} s (overlap {a.overlap})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
