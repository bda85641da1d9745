#!/bin/bash
# Texture reconstruction on the human: train, then evaluate on the test split and bake the
# texture -- the two steps of the reference's training_scripts/train_human_tex_recon.sh, run
# from a working directory holding configs/ and data/ (the reference's layout), through
# this build's train.py / eval.py.
#   bash training_scripts/train_human_tex_recon.sh intrinsic|tf+rff
set -e
method="$1"
PKG="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)/intrinsic-neural-fields_amd"
PY="${PYTHON:-python}"

if [ "$method" = "intrinsic" ]; then
    echo "Selected method: Intrinsic"
    CONFIG_PATH=configs/texture_reconstruction/intrinsic_human.yaml
    EVAL_OUT_DIR=out/texture_recon/intrinsic_human/test_eval
elif [ "$method" = "tf+rff" ]; then
    echo "Selected method: TF + RFF"
    CONFIG_PATH=configs/texture_reconstruction/tf_rff_human.yaml
    EVAL_OUT_DIR=out/texture_recon/tf_rff_human/test_eval
elif [ "$method" = "neutex" ]; then
    echo "NeuTex is outside this build's scope (see DESIGN.md)"
    exit 1
else
    echo "Unknown method: $method. Must be one of the following: tf+rff, neutex, intrinsic"
    exit 1
fi

"$PY" "$PKG/train.py" $CONFIG_PATH --allow_checkpoint_loading
"$PY" "$PKG/eval.py" $EVAL_OUT_DIR $CONFIG_PATH data/human_dataset_v2_tiny test --uv_mesh_path data/human_tri/RUST_3d_Low1.obj
