# A/B helper: run bench.py against another build of liblcpc_mi.so (argv[1]), e.g. one built from an
# older commit in a git worktree; the remaining arguments are bench.py's.
import os
import runpy
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lcpc_proof_of_storage_amd._native as N
N.load.__defaults__ = (sys.argv[1],)
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
