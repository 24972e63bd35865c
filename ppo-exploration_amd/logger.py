"""Key/value training logger with the reference's interface and CSV schema
(reference: logger.py:13-234 — record/dump/configure, stdout table, optional
CSV under ./logs/<ALGO>/<ENV>/run-<timestamp>.csv whose columns drop the
'prefix/' of each key and are extended when new keys appear)."""
import datetime
import os
import sys


class CSVWriter:
    def __init__(self, path):
        self.path = path
        self.keys = []
        self.rows = []

    def write(self, kv):
        flat = {}
        for k, v in kv.items():
            flat[k.split("/", 1)[1] if k.find("/") > 0 else k] = v
        new = [k for k in flat if k not in self.keys]
        if new:
            self.keys.extend(new)
        self.rows.append(flat)
        with open(self.path, "w") as f:  # rewrite: header grows with new keys
            f.write(",".join(self.keys) + "\n")
            for r in self.rows:
                f.write(",".join("" if r.get(k) is None else str(r.get(k)) for k in self.keys) + "\n")

    def close(self):
        pass


class TableWriter:
    def __init__(self, stream=sys.stdout):
        self.stream = stream

    def write(self, kv):
        if not kv:
            return
        items = [(str(k), f"{v:<8.3g}" if isinstance(v, float) else str(v)) for k, v in sorted(kv.items())]
        kw = max(len(k) for k, _ in items)
        vw = max(len(v) for _, v in items)
        bar = "-" * (kw + vw + 7)
        lines = [bar] + [f"| {k:<{kw}} | {v:<{vw}} |" for k, v in items] + [bar]
        self.stream.write("\n".join(lines) + "\n")
        self.stream.flush()

    def close(self):
        pass


class Logger:
    CURRENT = None

    def __init__(self, outputs, folder=None):
        self.outputs = outputs
        self.folder = folder
        self.kv = {}

    def record(self, key, value):
        self.kv[key] = value

    def dump(self, step=0):
        for o in self.outputs:
            o.write(dict(self.kv))
        self.kv.clear()


Logger.CURRENT = Logger([TableWriter()])


def record(key, value):
    Logger.CURRENT.record(key, value)


def dump(step=0):
    Logger.CURRENT.dump(step)


def get_values():
    return dict(Logger.CURRENT.kv)


def configure(algorithm, environment, log_to_file=False, folder=None, quiet=False):
    folder = os.path.join(folder or "./logs", algorithm, environment)
    outputs = [] if quiet else [TableWriter()]
    if log_to_file:
        os.makedirs(folder, exist_ok=True)
        name = "run" + datetime.datetime.now().strftime("-%Y-%m-%d-%H-%M-%S-%f") + ".csv"
        outputs.append(CSVWriter(os.path.join(folder, name)))
    Logger.CURRENT = Logger(outputs, folder=folder)
    if not quiet:
        print(f"Logging to {folder}")
