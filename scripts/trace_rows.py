"""Kernel dispatch rows of a rocprofv3 ``--kernel-trace`` run, from either output format.

rocprofv3 writes ``*_kernel_trace.csv`` with ``--output-format csv`` and a ``*_results.db`` SQLite file
(rocpd schema, the ``kernels`` view) by default. Both come back as dicts with the CSV column names the
summary scripts use: Start_Timestamp, End_Timestamp, Kernel_Name, Stream_Id, Queue_Id, Grid_Size_X/Y/Z,
Workgroup_Size_X, LDS_Block_Size, VGPR_Count.
"""
from __future__ import annotations

import csv
import gzip
import io
import sqlite3

_DB_COLS = {
    "Start_Timestamp": "start", "End_Timestamp": "end", "Kernel_Name": "name", "Stream_Id": "stream_id",
    "Queue_Id": "queue_id", "Grid_Size_X": "grid_x", "Grid_Size_Y": "grid_y", "Grid_Size_Z": "grid_z",
    "Workgroup_Size_X": "workgroup_x", "LDS_Block_Size": "lds_size", "VGPR_Count": "vgpr_count",
}


def load_rows(path: str) -> list[dict]:
    if path.endswith(".db"):
        con = sqlite3.connect(f"file:{path}?mode=ro", uri=True)
        try:
            sel = ", ".join(f"{v} AS {k}" for k, v in _DB_COLS.items())
            cur = con.execute(f"SELECT {sel} FROM kernels")
            names = [d[0] for d in cur.description]
            return [{k: ("" if v is None else str(v)) for k, v in zip(names, r)} for r in cur]
        finally:
            con.close()
    f = io.TextIOWrapper(gzip.open(path, "rb")) if path.endswith(".gz") else open(path)
    with f:
        return list(csv.DictReader(f))
