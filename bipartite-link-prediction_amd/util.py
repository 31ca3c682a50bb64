"""Drop-in for the reference's util.py (JSON score-file contract, progress logging).

Same names and behaviour as util.py:6-63, in Python 3. ``write_json`` writes the same
JSON text as ``json.dumps(d)`` (util.py:18-21): floats use Python's shortest round-trip
``repr``, ints stay ints -- the file contract eval.py:14 and the supervised_* scripts
read.
"""
import json
import subprocess
from time import time


def lines_in_file(fname):
    """Returns the number of lines in fname (util.py:6-9, shells out to wc -l)."""
    return int(subprocess.check_output(["wc", "-l", fname]).strip().split()[0])


def load_json(fname):
    """Reads the JSON data in fname and returns it as a dictionary (util.py:12-15)."""
    with open(fname) as f:
        return json.loads(f.read())


def write_json(d, fname):
    """Writes dictionary d to fname (util.py:18-21). A binary sidecar left beside an older
    version of the file is removed (it would describe the old scores)."""
    import os

    with open(fname, "w") as f:
        f.write(json.dumps(d))
    if os.path.exists(fname + ".npz"):
        os.unlink(fname + ".npz")


def write_sidecar(d, fname):
    """Binary sidecar of a score file: ``fname + '.npz'`` with the same pairs and values as
    ``write_json(d, fname)``: int64 ``users`` / ``businesses``, float64
    ``scores`` and a bool ``is_int`` (JSON ints: CN counts and the reference's int 0s), in
    the dict's order. Loads in milliseconds where json.loads of million-pair files takes
    seconds; ``load_scores`` reads it back as the same dict. The sidecar records the size
    and mtime of the JSON it describes (``json_stat``): ``load_scores`` ignores it once the
    JSON has been rewritten by anything else (e.g. the reference's own scripts)."""
    import os

    import numpy as np

    us, bs, vals, ints = [], [], [], []
    for u, inner in d.items():
        for b, v in inner.items():
            us.append(int(u))
            bs.append(int(b))
            vals.append(float(v))
            ints.append(isinstance(v, int) and not isinstance(v, bool))
    np.savez(fname + ".npz", users=np.array(us, np.int64), businesses=np.array(bs, np.int64),
             scores=np.array(vals, np.float64), is_int=np.array(ints, bool), json_stat=_json_stat(fname))


def _json_stat(fname):
    import os

    import numpy as np

    if not os.path.exists(fname):
        return np.array([-1, -1], np.int64)
    st = os.stat(fname)
    return np.array([st.st_size, st.st_mtime_ns], np.int64)


def load_scores(fname):
    """The score dict of ``fname``: from its binary sidecar when present, else the JSON."""
    import os

    import numpy as np

    side = fname + ".npz"
    if not os.path.exists(side):
        return load_json(fname)
    z = np.load(side)
    if os.path.exists(fname) and ("json_stat" not in z.files or
                                  not np.array_equal(z["json_stat"], _json_stat(fname))):
        return load_json(fname)  # stale: the JSON changed after the sidecar was written
    out = {}
    for u, b, v, i in zip(z["users"].tolist(), z["businesses"].tolist(), z["scores"].tolist(), z["is_int"].tolist()):
        out.setdefault(str(u), {})[str(b)] = int(v) if i else v
    return out


def load_json_lines(fname):
    """Yields one JSON object per line of fname (util.py:24-28)."""
    with open(fname) as f:
        for line in f:
            yield json.loads(line)


class LoopLogger:
    """Prints the progress of an iteration (util.py:31-55)."""

    def __init__(self, step_size, size=0, print_time=False):
        self.step_size = step_size
        self.size = size
        self.n = 0
        self.print_time = print_time

    def step(self):
        if self.n == 0:
            self.start_time = time()
        self.n += 1
        if self.n % self.step_size == 0:
            if self.size == 0:
                print("On item " + str(self.n))
            else:
                line = "{:}/{:}, {:.1f}%,".format(self.n, self.size, 100.0 * self.n / self.size)
                if self.print_time:
                    elapsed = time() - self.start_time
                    line += " elapsed: {:.1f}s,".format(elapsed)
                    line += " remaining: {:.1f}s".format((self.size - self.n) * elapsed / self.n)
                print(line)


def logged_loop(iterable, loop_logger):
    """Iterate through iterable while printing progress with loop_logger (util.py:58-63)."""
    loop_logger.n = 0
    for elem in iterable:
        loop_logger.step()
        yield elem
