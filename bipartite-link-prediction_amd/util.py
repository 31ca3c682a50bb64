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
    """Writes dictionary d to fname (util.py:18-21)."""
    with open(fname, "w") as f:
        f.write(json.dumps(d))


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
