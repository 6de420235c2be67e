"""Run a script with faulthandler dumping every thread's Python stack every 30 s to
stderr (diagnosing a silent multi-rank run). Usage: trace_run.py SCRIPT ARGS..."""
import faulthandler
import runpy
import sys

faulthandler.dump_traceback_later(30, repeat=True)
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
