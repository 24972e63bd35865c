"""Logger parity (reference logger.py:13-234) against the reference's
own output: tests/golden/logger.npz holds the CSV file and stdout tables the reference
logger wrote for three dumps whose later ones bring new keys (make_golden.py gen_logger)."""
import ast
import csv
import io
import os

import numpy as np

import logger


def _dumps(f):
    return [dict(zip(f[f"d{i}_keys"].tolist(), [ast.literal_eval(v) for v in f[f"d{i}_vals"].tolist()]))
            for i in range(int(f["n_dumps"]))]


def _rows(text):
    r = list(csv.reader(io.StringIO(text)))
    header, body = r[0], r[1:]
    return header, [dict(zip(header, row)) for row in body]


def test_csv_and_table_match_reference(golden, tmp_path):
    f = golden("logger")
    buf = io.StringIO()
    logger.configure("PPO", "Fake-v0", log_to_file=True, folder=str(tmp_path), quiet=True)
    logger.Logger.CURRENT.outputs.insert(0, logger.TableWriter(buf))
    tables = []
    for kv in _dumps(f):
        start = len(buf.getvalue())
        for k, v in kv.items():
            logger.record(k, v)
        logger.dump(step=0)
        tables.append(buf.getvalue()[start:])
    folder = tmp_path / "PPO" / "Fake-v0"
    (name,) = os.listdir(folder)
    assert name.startswith("run-") and name.endswith(".csv")
    logger.configure("PPO", "Fake-v0", quiet=True)  # closes the CSV
    text = (folder / name).read_text()
    h_ref, rows_ref = _rows(str(f["csv"]))
    h, rows = _rows(text)
    # same columns (the reference appends new ones in hash-set order, which varies per run)
    assert sorted(h) == sorted(h_ref) and len(h) == len(h_ref)
    assert rows == rows_ref
    assert tables[0] == str(f["table0"]) and tables[1] == str(f["table1"])


def test_csv_rewrites_header_once_per_new_key_set(tmp_path):
    w = logger.CSVWriter(str(tmp_path / "a.csv"))
    w.write({"time/x": 1})
    w.write({"time/x": 2})
    w.write({"time/x": 3, "train/y": 0.5})
    w.write({"time/x": 4, "train/y": 0.25, "train/z": 7})
    assert not hasattr(w, "rows")  # earlier rows are re-read from the file, not held
    w.close()
    assert (tmp_path / "a.csv").read_text() == "x,y,z\n1,,\n2,,\n3,0.5,\n4,0.25,7\n"
