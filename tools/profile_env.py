"""cProfile of one VecAHRAGGymEnv reset + episode on the C5 workload (diagnostic).

Runs tools/bench_env.py's workload and profiles the second reset (warm: device graph, index and
host caches built) and the steps that follow; prints the top functions by cumulative time.
"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools")]

import bench_env  # noqa: E402


def main():
    sys.argv = ["bench_env.py", "--envs", "1024", "--steps", "6", "--single", "4"]
    prof = {"reset": cProfile.Profile(), "step": cProfile.Profile()}
    calls = {"reset": 0, "step": 0}

    def wrap(name):
        orig = getattr(bench_env.VecAHRAGGymEnv, name)

        def f(self, *a, **k):
            calls[name] += 1
            if (name == "reset" and calls[name] == 2) or (name == "step" and calls["reset"] == 2):
                prof[name].enable()
                try:
                    return orig(self, *a, **k)
                finally:
                    prof[name].disable()
            return orig(self, *a, **k)
        setattr(bench_env.VecAHRAGGymEnv, name, f)

    wrap("reset")
    wrap("step")
    bench_env.main()
    for name, p in prof.items():
        s = io.StringIO()
        pstats.Stats(p, stream=s).sort_stats("tottime").print_stats(25)
        print(f"==== {name} (by own time)\n" + s.getvalue()[:5000])


if __name__ == "__main__":
    main()
