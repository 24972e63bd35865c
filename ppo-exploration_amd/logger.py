"""Key/value training logger with the reference's interface and CSV schema
(reference: logger.py:13-234 — record/dump/configure, stdout table, optional
CSV under ./logs/<ALGO>/<ENV>/run-<timestamp>.csv whose columns drop the
'prefix/' of each key and are extended when new keys appear)."""
import datetime
import os
import sys


class CSVWriter:
    """CSV rows of the dumped key/values (logger.py:13-58): a key's 'prefix/' is dropped
    (its second '/'-separated field is the column), columns are appended when new keys
    appear — the file is re-read, rewritten with the wider header and the earlier rows padded
    with one empty field per new column, as the reference does (no rows held in memory) — and
    every dump appends one row.  The reference appends new columns in set order (hash order:
    it varies from run to run); here in first-seen order."""

    def __init__(self, path):
        self.path = path
        self.keys = []
        self.file = open(path, "w+t")

    @staticmethod
    def _line(keys, row):
        return ",".join("" if row.get(k) is None else str(row.get(k)) for k in keys) + "\n"

    def write(self, kv):
        flat = {}
        for k, v in kv.items():
            flat[k.split("/")[1] if k.find("/") > 0 else k] = v
        new = [k for k in flat if k not in self.keys]
        if new:
            self.keys.extend(new)
            self.file.seek(0)
            lines = self.file.readlines()
            self.file.seek(0)
            self.file.truncate()
            self.file.write(",".join(self.keys) + "\n")
            for line in lines[1:]:
                self.file.write(line[:-1] + "," * len(new) + "\n")
        self.file.write(self._line(self.keys, flat))
        self.file.flush()

    def close(self):
        self.file.close()


class TableWriter:
    """The stdout table (logger.py:61-130): keys sorted, grouped under their 'tag/' header
    rows, names and values truncated to 23 characters, floats as {:<8.3g}."""

    def __init__(self, stream=None):
        self.stream = stream if stream is not None else sys.stdout

    @staticmethod
    def _truncate(s, max_length=23):
        return s[: max_length - 3] + "..." if len(s) > max_length else s

    def write(self, kv):
        key2str = {}
        tag = None
        for key, value in sorted(kv.items()):
            value_str = f"{value:<8.3g}" if isinstance(value, float) else str(value)
            if key.find("/") > 0:
                tag = key[: key.find("/") + 1]
                key2str[self._truncate(tag)] = ""
            if tag is not None and tag in key:
                key = "   " + key[len(tag):]
            key2str[self._truncate(key)] = self._truncate(value_str)
        if not key2str:
            return
        kw = max(map(len, key2str.keys()))
        vw = max(map(len, key2str.values()))
        dashes = "-" * (kw + vw + 7)
        lines = [dashes] + [f"| {k}{' ' * (kw - len(k))} | {v}{' ' * (vw - len(v))} |" for k, v in key2str.items()]
        lines.append(dashes)
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

    def get_dir(self):
        return self.folder

    def close(self):
        for o in self.outputs:
            o.close()


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
    if Logger.CURRENT is not None:
        Logger.CURRENT.close()  # a reconfigure ends the previous run's CSV file
    Logger.CURRENT = Logger(outputs, folder=folder)
    if not quiet:
        print(f"Logging to {folder}")
