"""Device plumbing: torch-ROCm supplies HBM buffers and the current HIP stream.

Torch is plumbing only — every compute step on the hot path is a libmjx HIP
kernel called through the C ABI.
"""
import numpy as np
import torch

from ._lib import MjxError, MJX_I8, MJX_I32, MJX_I64

_DTYPE_CODE = {torch.int8: MJX_I8, torch.int32: MJX_I32, torch.int64: MJX_I64}


def require_gpu():
    if not torch.cuda.is_available():
        raise MjxError("no HIP device visible: the majority-dynamics kernels run only on the GPU "
                       "(gfx950); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def cu_count():
    """Compute units of the current device (256 on an MI355X)."""
    return torch.cuda.get_device_properties(require_gpu()).multi_processor_count


def stream_handle():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise MjxError("expected a device tensor")
    if not t.is_contiguous():
        raise MjxError("expected a contiguous tensor")
    return t.data_ptr()


def dtype_code(t):
    try:
        return _DTYPE_CODE[t.dtype]
    except KeyError:
        raise MjxError(f"spin arrays must be int8/int32/int64, got {t.dtype}") from None


def to_device(x, dtype=None):
    """numpy array or tensor -> contiguous device tensor (optionally cast)."""
    dev = require_gpu()
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x))
    elif isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.as_tensor(np.asarray(x))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.to(dev).contiguous()


def words_for(R):
    return (int(R) + 63) // 64
