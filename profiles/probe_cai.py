"""Probe (GPU box): does torch-ROCm wrap foreign device memory through __cuda_array_interface__?"""
import torch


class DevArray:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {'shape': (n,), 'typestr': '<i8', 'data': (ptr, False), 'version': 2,
                                         'strides': None}


a = torch.arange(1000, dtype=torch.int64, device='cuda')
v = torch.as_tensor(DevArray(a.data_ptr() + 8 * 10, 20), device='cuda')
print('cai ok', v.device, v.dtype, v.shape, v[:3].tolist(), v.data_ptr() == a.data_ptr() + 80)
