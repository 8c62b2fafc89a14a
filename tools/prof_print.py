#!/usr/bin/env python3
"""Print a cProfile dump sorted by own time: python tools/prof_print.py DUMP [N]."""
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
