"""Named configurations (SURVEY.md §8d / BASELINE.json `configs`), all expressed through
the reference's own `create_vision_transformer_detector` kwargs (vtd.py:498-506)."""

# C1: the reference default (notebook config, ipynb:394-403), 608x608, patch 17, D 28.
C1_REFERENCE_DEFAULT = dict(input_shape=(608, 608, 3))

# C2: "ViT-B/16 @224".  ViT-B's 768->3072->768 MLP is not expressible with the reference's
# pyramid `D * 2**(q-1..0)` (vtd.py:385-386); q = 3 gives 768->3072->1536->768 (the closest
# that contains the 3072 hidden layer).  GELU(tanh) per north_star; default 7-layer head.
VIT_B16_224 = dict(input_shape=(224, 224, 3), patch_size=16, embedding_dim=768,
                   encoder_num_heads=12, encoder_key_dim=64, encoder_repeat_times=12,
                   encoder_mlp_quantities=3, use_mish=False, mlp_head_last_units=136,
                   mlp_head_dense_layers_quantity=7)

# C3: ViT-B/16 at 640x640 (1600 tokens, long-sequence attention).
VIT_B16_640 = dict(VIT_B16_224, input_shape=(640, 640, 3))

# C5: ViT-L/16 @384.
VIT_L16_384 = dict(input_shape=(384, 384, 3), patch_size=16, embedding_dim=1024,
                   encoder_num_heads=16, encoder_key_dim=64, encoder_repeat_times=24,
                   encoder_mlp_quantities=3, use_mish=False, mlp_head_last_units=136,
                   mlp_head_dense_layers_quantity=7)

PRESETS = {"c1": C1_REFERENCE_DEFAULT, "vit_b16_224": VIT_B16_224,
           "vit_b16_640": VIT_B16_640, "vit_l16_384": VIT_L16_384}
