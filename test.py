"""Reference-compatible evaluation entry point (``python test.py --flags``)."""
from cst_captioning_amd.cli import test_main

if __name__ == '__main__':
    test_main()
