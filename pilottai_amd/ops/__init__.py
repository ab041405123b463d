"""CDNA4 kernels (HIP, gfx950) and their fp32 PyTorch references."""
from .kernels import (  # noqa: F401
    cosine_topk,
    decode_gemm,
    decode_qkv_rope,
    wide_gemm,
    wide_workspace,
    pack_decode_qkv_rope,
    pack_decode_gate_up,
    pack_decode_weight,
    fused_add_rmsnorm,
    linear,
    native_available,
    native_module_path,
    paged_attention,
    require_native,
    rmsnorm,
    rope_cache,
    sample,
    sample_workspace,
    topkp_threshold,
    silu_mul,
    skinny_gemm,
    SKINNY_MAX_M,
)
from .attn_meta import ATT_PART, build_attention_items  # noqa: F401
from . import reference  # noqa: F401
