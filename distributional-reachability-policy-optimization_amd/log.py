"""Run log and CSV tables with the reference's file formats (src/log.py:6-73).

``default_log`` is the process-wide text log. When a driver has already set up
the reference's own ``src.log.default_log`` (main.py through src/cli.py), this
one follows it, so the trainer's ``episodes.csv`` lands in the same run
directory and ``log.message`` goes to the same ``log.txt``."""
import csv
import sys
from datetime import datetime
from pathlib import Path


class Log:
    def __init__(self):
        self._dir = None
        self._log_file = None

    def _delegate(self):
        if self._dir is not None:
            return None
        ref = sys.modules.get('src.log')
        other = getattr(ref, 'default_log', None) if ref is not None else None
        if other is not None and other is not self and getattr(other, 'dir', None) is not None:
            return other
        return None

    def setup(self, dir, log_filename='log.txt', if_exists='append'):
        self._dir = Path(dir)
        self._dir.mkdir(exist_ok=True)
        path = self._dir / log_filename
        if path.exists() and if_exists == 'exit':
            print(f'Log file named {log_filename} already exists; exiting')
            sys.exit()
        if path.exists() and if_exists not in ('append', 'overwrite'):
            raise NotImplementedError(f'Unknown if_exists option: {if_exists}')
        mode = 'a' if (path.exists() and if_exists == 'append') else 'w'
        self._log_file = path.open(mode, buffering=1)

    @property
    def dir(self):
        d = self._delegate()
        return d.dir if d is not None else self._dir

    def message(self, message, timestamp=True, flush=False):
        d = self._delegate()
        if d is not None:
            return d.message(message, timestamp=timestamp, flush=flush)
        if timestamp:
            message = f'[{datetime.now().strftime("%H:%M:%S")}] ' + message
        else:
            message = ' ' * 11 + message
        print(message)
        if self._log_file is not None:
            self._log_file.write(f'{message}\n')
            if flush:
                self._log_file.flush()

    def __call__(self, *args, **kwargs):
        return self.message(*args, **kwargs)


default_log = Log()


class TabularLog:
    """Append-mode CSV whose header is the first row's keys (src/log.py:55-73)."""

    def __init__(self, dir, filename):
        self._dir = Path(dir)
        assert self._dir.is_dir()
        self._filename = filename
        self._column_names = None
        self._file = open(self.path, mode=('a' if self.path.exists() else 'w'), newline='')
        self._writer = csv.writer(self._file)

    @property
    def path(self):
        return self._dir / self._filename

    def row(self, row, flush=True):
        if self._column_names is None:
            self._column_names = list(row.keys())
            self._writer.writerow(self._column_names)
        self._writer.writerow([row[c] for c in self._column_names])
        if flush:
            self._file.flush()
