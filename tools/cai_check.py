"""Can torch wrap a device buffer it did not allocate (diagnostic)?
__cuda_array_interface__ and CUDAPluggableAllocator + MemPool, on
hipExtMallocWithFlags(hipDeviceMallocUncached) memory."""
import ctypes
import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
p = ctypes.c_void_p()
rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(3))
print("hipExtMallocWithFlags rc", rc, hex(p.value or 0))


class Buf:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 2,
                                         "strides": None}


try:
    t = torch.as_tensor(Buf(p.value, 1 << 20), device="cuda")
    t.fill_(7)
    torch.cuda.synchronize()
    print("as_tensor ok", t.data_ptr() == p.value, int(t.sum()), t.device)
except Exception as e:  # noqa: BLE001
    print("as_tensor failed:", type(e).__name__, e)
