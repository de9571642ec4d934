#!/usr/bin/env python3
"""A tool to bruteforce fastest winning moves for the board game Splendor — on MI355X.

Drop-in for the reference CLI (same flags and output) with the beam search on the GPU engine.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from splendor_amd.cli import cli  # noqa: E402

if __name__ == '__main__':
    cli()
