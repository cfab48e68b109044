"""experiment runner: bench.py against an alternative engine library"""
import sys
sys.path.insert(0, '/root/repo')
from shadow_amd import engine as E
E.LIB_PATH = sys.argv[1]
import bench
sys.argv = ['bench.py'] + sys.argv[2:]
bench.main()
