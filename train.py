"""Reference-compatible training entry point (``python train.py --flags``)."""
from cst_captioning_amd.cli import train_main

if __name__ == '__main__':
    train_main()
