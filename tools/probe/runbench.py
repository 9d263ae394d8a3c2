import sys, runpy, atexit
atexit.register(lambda: print("[atexit]", file=sys.stderr, flush=True))
sys.argv = ["bench.py"] + sys.argv[1:]
try:
    runpy.run_path("bench.py", run_name="__main__")
except SystemExit as e:
    print("[sysexit]", e.code, file=sys.stderr, flush=True); raise
except BaseException:
    import traceback; traceback.print_exc(); raise
print("[done]", file=sys.stderr, flush=True)
