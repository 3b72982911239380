import ctypes as C, sys
sys.path.insert(0, '/root/repo')
from broadway_amd import _lib
L = _lib.mi()
import torch; torch.cuda.init()
a, b, c, d = (C.c_int() for _ in range(4))
print("rc", L.h264mi_kernel_occupancy(C.byref(a), C.byref(b), C.byref(c), C.byref(d)), "blocks/CU", a.value, "lds", b.value, "regs", c.value)
p = torch.cuda.get_device_properties(0)
print(p.multi_processor_count, getattr(p, "shared_memory_per_multiprocessor", None), getattr(p, "max_threads_per_multi_processor", None))
