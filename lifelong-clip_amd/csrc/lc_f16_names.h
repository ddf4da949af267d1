// Included first (-include) in the IEEE-half objects of the 16-bit kernel sources (make: the
// build/f16_*.o objects, -DLC_F16): every external symbol of those sources gets the suffix _f16,
// so both storage types link into one liblcclip.so. include/lc_clip.h declares the _f16 entry
// points the text tower uses.
#pragma once
#define lc_attn_fwd lc_attn_fwd_f16
#define lc_attn_bwd_fp8 lc_attn_bwd_fp8_f16
#define lc_attn_bwd lc_attn_bwd_f16
#define lc_attn_bwd_set_form lc_attn_bwd_set_form_f16
#define lc_gemm_nt_ex lc_gemm_nt_ex_f16
#define lc_gemm_nt lc_gemm_nt_f16
#define lc_gemm_nt_ws lc_gemm_nt_ws_f16
#define lc_gemm_set_debug lc_gemm_set_debug_f16
#define lc_gemm_nt_fp8 lc_gemm_nt_fp8_f16
#define lc_gemm_set_tile lc_gemm_set_tile_f16
#define lc_gemm_set_streamk lc_gemm_set_streamk_f16
#define lc_gemm_tn lc_gemm_tn_f16
#define lc_gemm_tn_ws lc_gemm_tn_ws_f16
#define lc_adapter_wgrad lc_adapter_wgrad_f16
#define lc_adapter_wgrad_ws lc_adapter_wgrad_ws_f16
#define lc_layernorm_fwd lc_layernorm_fwd_f16
#define lc_layernorm_fwd_fp8 lc_layernorm_fwd_fp8_f16
#define lc_layernorm_bwd lc_layernorm_bwd_f16
#define lc_layernorm_bwd_fp8 lc_layernorm_bwd_fp8_f16
#define lc_patchify lc_patchify_f16
#define lc_vit_assemble lc_vit_assemble_f16
#define lc_vit_embed_ln lc_vit_embed_ln_f16
#define lc_text_embed lc_text_embed_f16
#define lc_eot_rows lc_eot_rows_f16
#define lc_cast_bf16 lc_cast_bf16_f16
#define lc_merge_weight lc_merge_weight_f16
#define lc_cast_weights_bf16 lc_cast_weights_bf16_f16
#define lc_merge_weights_bf16 lc_merge_weights_bf16_f16
#define lc_lora_grad lc_lora_grad_f16
#define lc_lora_grad_ws lc_lora_grad_ws_f16
#define lc_adapter_fwd lc_adapter_fwd_f16
#define lc_adapter_ln_fwd lc_adapter_ln_fwd_f16
#define lc_adapter_bwd_set_form lc_adapter_bwd_set_form_f16
#define lc_adapter_bwd lc_adapter_bwd_f16
#define lc_check_finite lc_check_finite_f16
#define lc_adamw lc_adamw_f16
#define lc_counter_add lc_counter_add_f16
#define lc_adam_step_advance lc_adam_step_advance_f16
