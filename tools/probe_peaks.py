import sys, json
sys.path.insert(0, '.')
import bench_kernels as bk
print(json.dumps(bk.probe_peaks(), indent=1))
