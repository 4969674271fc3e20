"""Configuration for the MI355X-native captioning train path.

Same module-level names and defaults as the reference's config.py (config.py:1-145) so code written
against the reference keeps working; additions for this build are grouped at the end
(MEMORY_MODE, DTYPE, ENCODER_SPECS, ...).
"""
import os

import torch

# --- General (reference config.py:10-12) ---
DEVICE = "cuda" if torch.cuda.is_available() else "cpu"
RANDOM_SEED = 42

# --- Data (reference config.py:17-35) ---
DATA_DIR = os.environ.get("MIT_DATA_DIR", "../assets/multimodal_image_transformer/")
IMAGE_DIR = DATA_DIR + "images"
CAPTIONS_FILE = DATA_DIR + "captions.json"
OUTPUT_DIR = DATA_DIR
TRAIN_SPLIT_RATIO = 0.9
NUM_WORKERS = 2
PIN_MEMORY = DEVICE == "cuda"

# --- Model (reference config.py:41-72) ---
ENCODER_MODEL_NAME = "google/vit-base-patch16-224-in21k"
IMAGE_PROCESSOR_NAME = "google/vit-base-patch16-224-in21k"
IMG_TRANSFORM_MODE = "hf_processor"
VOCAB_SIZE = 10000
MAX_SEQ_LEN = 100
DECODER_EMBED_DIM = 512
DECODER_LAYERS = 6
DECODER_HEADS = 8
DECODER_FF_DIM = 2048
DECODER_DROPOUT = 0.1
PROJECTION_DIM = 512

# --- Training (reference config.py:76-100) ---
BATCH_SIZE = 32
NUM_EPOCHS = 20
LEARNING_RATE = 1e-4
WEIGHT_DECAY = 1e-5
GRAD_CLIP_VALUE = 5.0
ADAM_BETA1 = 0.9
ADAM_BETA2 = 0.98
ADAM_EPS = 1e-9
WARMUP_STEPS = 0
LOG_INTERVAL = 50
VALIDATION_INTERVAL = 1
CHECKPOINT_PREFIX = "model_checkpoint"
RESUME_CHECKPOINT_PATH = None

# --- Tokenizer (reference config.py:110-123) ---
PAD_TOKEN = "<PAD>"
START_TOKEN = "<START>"
END_TOKEN = "<END>"
UNK_TOKEN = "<UNK>"
PAD_TOKEN_ID = 0
START_TOKEN_ID = 1
END_TOKEN_ID = 2
UNK_TOKEN_ID = 3
VOCAB_PATH = OUTPUT_DIR + "vocab.json"
MERGES_PATH = OUTPUT_DIR + "merges.txt"

# --- Inference (reference config.py:137) ---
BEAM_SIZE = 3

# =====================================================================================
# Additions of this build
# =====================================================================================
# Decoder memory: "cls" = the reference model.py:141-151 behaviour (CLS token only, S = 1);
# "patches" = cross-attention over the whole projected patch sequence (BASELINE north star).
MEMORY_MODE = os.environ.get("MIT_MEMORY_MODE", "cls")
# Compute dtype of activations / GEMM operands: "bf16" (fp32 accumulation; fp32 master weights,
# grads and AdamW state) or "fp32" (parity mode: fp32 end to end).
DTYPE = os.environ.get("MIT_DTYPE", "bf16")
# Local weights for the frozen encoder (HF state_dict names, .safetensors). There is no network, so
# from_pretrained(ENCODER_MODEL_NAME) is replaced by this file; None -> seeded random init.
ENCODER_WEIGHTS_PATH = os.environ.get("MIT_ENCODER_WEIGHTS", None)
# bf16 encoders: keep the residual stream in f32 (as torch.autocast does; the sublayer outputs stay
# bf16). "auto" = the 24-layer CLIP-L towers (configs[2] / configs[3]), where a bf16 stream doubles
# the encoder's error; "on" / "off" force it.
ENCODER_F32_RESIDUAL = os.environ.get("MIT_ENCODER_F32_RESIDUAL", "auto")
# bf16 ViT towers on the bf16 stream: fold each pre-LN LayerNorm into the GEMM that consumes it
# (encoder.fold_layernorm). "auto" = on where it applies; "off" keeps the explicit LayerNorm launches.
ENCODER_FOLD_LN = os.environ.get("MIT_ENCODER_FOLD_LN", "auto")
# A NaN / inf training loss (e.g. an all-PAD batch): "warn" (default; the reference trains on through it)
# reports the first such batch of the epoch, "raise" stops train_one_epoch with NonFiniteLossError.
NONFINITE_LOSS = os.environ.get("MIT_NONFINITE_LOSS", "warn")

# Encoder geometry by model name (values of the HF configs the names resolve to).
ENCODER_SPECS = {
    "google/vit-base-patch16-224-in21k": dict(kind="vit", hidden=768, layers=12, heads=12, mlp=3072, image=224,
                                              patch=16, eps=1e-12),
    "google/vit-base-patch16-224": dict(kind="vit", hidden=768, layers=12, heads=12, mlp=3072, image=224, patch=16,
                                        eps=1e-12),
    "openai/clip-vit-base-patch32": dict(kind="clip", hidden=768, layers=12, heads=12, mlp=3072, image=224, patch=32,
                                         eps=1e-5),
    "openai/clip-vit-base-patch16": dict(kind="clip", hidden=768, layers=12, heads=12, mlp=3072, image=224, patch=16,
                                         eps=1e-5),
    "openai/clip-vit-large-patch14": dict(kind="clip", hidden=1024, layers=24, heads=16, mlp=4096, image=224,
                                          patch=14, eps=1e-5),
    "openai/clip-vit-large-patch14-336": dict(kind="clip", hidden=1024, layers=24, heads=16, mlp=4096, image=336,
                                              patch=14, eps=1e-5),
}
