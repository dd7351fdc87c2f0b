"""ctypes signatures of the C ABI exported by ``libmi355x_kernels.so``.

One entry per ``MI_API`` function in ``csrc/kernels/*.hip``.
"""
from ._lib import signature, c_void_p as P, c_int as I, c_int64 as L, c_float as F
import ctypes

U32 = ctypes.c_uint32

# gemm_conv.hip
signature("mi_conv2d_fwd", P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_nt_stat_rows", I, I)
signature("mi_set_glds", I)
signature("mi_set_nt_stages", I)
signature("mi_set_nt_split_blocks", I)
signature("mi_set_nt_split_fused", I)
signature("mi_set_tn_split_fused", I)
signature("mi_conv2d_dgrad", P, P, P, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_conv2d_wgrad", P, P, P, I, I, I, I, I, I, I, I, I, I, I, P)
# normalize-on-load of inner BatchNorms (ops/resblock.py)
signature("mi_conv_nol_ok", I, I, I, I, I, I, I, I, I, I, I)
signature("mi_conv2d_fwd_nol", P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_conv2d_wgrad_nol", P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_conv2d_dgrad_ex3", P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, I, P, I, P, P, P)
signature("mi_conv2d_dgrad_ex4", P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, I, P, I, P, P, P, P)
signature("mi_conv_wtrans", P, P, I, I, I, P)
# stem_conv.hip (ops/stem.py): weight pack and the gradient straight into the parameter's buffer
signature("mi_stem_wpack", P, P, I, I, I, I, L, L, L, L, P)
signature("mi_stem_wgrad_to", P, P, P, I, L, L, L, L, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_conv_wtrans_multi", P, P, P, I, I, P)
signature("mi_gemm_nt", P, P, P, P, P, I, I, I, I, I, I, I, I, P)
signature("mi_gemm_tn", P, P, P, I, I, I, I, I, I, P)
signature("mi_gemm_tn_bias", P, P, P, P, I, I, I, I, I, I, P)
signature("mi_register_wgrad_stream", P)
signature("mi_register_aux_stream", P)
signature("mi_create_cu_masked_stream", I, I, P)
signature("mi_splitk_ws_reserve", ctypes.c_size_t, P)

# norm_act.hip
signature("mi_bn_partial_rows", I, I)
signature("mi_bn_slab_extra_rows")
signature("mi_bn_set_small_elems", L)
signature("mi_bn_init_counters")
signature("mi_bn_fwd_train", P, P, P, I, I, F, F, P, P, P, P, P, P, P, P, P, P, I, I, P)
signature("mi_bn_apply_dual", P, P, P, I, I, P, P, P, P, I, P)
signature("mi_bn_apply_bits", P, P, P, P, I, I, P, P, P, P, P)
signature("mi_bn_fwd_eval", P, P, P, I, I, F, P, P, P, P, P, P, I, P)
signature("mi_bn_bwd_train", P, P, P, P, P, I, I, P, P, P, P, P, P, P, I, P)
signature("mi_bn_bwd_eval", P, P, P, P, P, I, I, I, P)
signature("mi_bnpool_partial_rows", I, I)
signature("mi_bnpool_fwd", P, P, P, P, P, I, I, I, I, I, I, I, I, I, P)
signature("mi_bnpool_bwd", P, P, P, P, I, I, I, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P)

# misc.hip
signature("mi_maxpool_fwd", P, P, P, I, I, I, I, I, I, I, I, I, P)
signature("mi_maxpool_bwd", P, P, P, I, I, I, I, I, I, I, I, I, P)
signature("mi_gap_fwd", P, P, I, I, I, P)
signature("mi_gap_bwd", P, P, I, I, I, P)
signature("mi_ce_fwd", P, P, P, P, I, I, I, P)
signature("mi_ce_bwd", P, P, P, P, P, I, I, I, I, I, P)
signature("mi_sgd_flat", P, P, P, P, L, F, F, F, F, I, I, F, P)
signature("mi_cast_bf16", P, P, L, P)
signature("mi_augment", P, P, I, I, I, I, I, I, I, U32, P, P, P)
signature("mi_im2col", P, P, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_add_bf16", P, P, P, L, P)
signature("mi_checksum", P, L, P, P)
signature("mi_flags_alloc", I, P)
signature("mi_flag_bump", P, P)
signature("mi_flag_gate", P, U32, P, I, P)
signature("mi_host_word_alloc", P, P)
signature("mi_capture_enter", restype=None)
signature("mi_capture_exit", restype=None)
signature("mi_capture_depth")

# gemm_conv.hip (epilogue-fused NT GEMM)
signature("mi_gemm_nt_epi", P, P, P, P, P, I, I, I, I, I, I, I, P)

# transformer.hip
signature("mi_layernorm_fwd", P, P, P, P, P, P, I, I, F, P)
signature("mi_layernorm_bwd", P, P, P, P, P, P, P, P, P, I, I, P)
signature("mi_colsum_bf16", P, P, I, I, I, P)
signature("mi_vit_patchify", P, P, I, I, I, I, I, I, P)
signature("mi_vit_embed_fwd", P, P, P, P, I, I, I, P)
signature("mi_vit_embed_bwd_part_floats", I, I, I, restype=L)
signature("mi_vit_embed_bwd", P, P, P, P, P, I, I, I, P)
signature("mi_cast_colsum_f32", P, P, P, I, I, P)
signature("mi_ln_ws_reserve", I, P)

# attention.hip
signature("mi_attn_max_seq")
signature("mi_attn_fwd", P, P, P, I, I, I, F, P)
signature("mi_attn_bwd", P, P, P, P, P, P, I, I, I, F, P)
signature("mi_set_att_waves", I)

# gemm256.hip
signature("mi_gemm256_nt", P, P, P, P, P, I, I, I, I, I, I, I, I, I, P)
signature("mi_gemm256p_nt", P, P, P, P, P, I, I, I, I, I, I, I, P)
signature("mi_set_gemm_persist", I)
signature("mi_set_tail_split", I)
signature("mi_set_gemm256", I)
signature("mi_g256_tail_ws_reserve", ctypes.c_size_t, I, P)
signature("mi_gemm256_tn", P, P, P, I, I, I, I, I, I, P)
signature("mi_dgrad_stat_rows", I, I, I, I, I, I, I, I, I)
signature("mi_conv_stat_rows", I, I, I, I)
signature("mi_conv_stat_rows_g", I, I, I, I, I, I, I, I, I, I, I)
signature("mi_gemm256_conv", I, P, P, P, P, I, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P)
signature("mi_conv2d_dgrad_ex", P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, I, P, P)
signature("mi_conv2d_dgrad_ex2", P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P, P, I, P, I, P)
signature("mi_bn_bwd_train_pre", P, P, P, P, I, I, P, P, P, P, P, P, P, I, P)
signature("mi_set_conv256_min_tiles", I)
signature("mi_set_conv256_min_k", I)
