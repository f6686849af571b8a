#!/usr/bin/env python3
"""Run one of the reference's entry scripts (main.py, parallel_main.py) with
this repository's ``model`` / ``train`` packages in place of the reference's.

    python tools/ref_entry.py /path/to/reference/main.py config.yml da-vinci ...

Python puts a script's own directory first on sys.path, which would pick the
reference's ``model``/``train``; this stub puts uncertainty-model_amd/ in
front, keeps the reference directory behind it (for ``loaders``), changes
into the reference directory (its config and graph paths are CWD-relative)
and runs the script in this same process (runpy, no exec).
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'uncertainty-model_amd')


def main():
    if len(sys.argv) < 2:
        sys.exit(__doc__)
    script = os.path.abspath(sys.argv[1])
    ref_dir = os.path.dirname(script)
    sys.argv = [script] + sys.argv[2:]
    sys.path[:0] = [PKG, ref_dir]
    os.chdir(ref_dir)
    runpy.run_path(script, run_name='__main__')


if __name__ == '__main__':
    main()
