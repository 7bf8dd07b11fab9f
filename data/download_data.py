"""Download the raw LendingClub data (reference: data/download_data.py)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from cobalt_smart_lender_ai_amd.dataio.datasets import download_data  # noqa: E402

if __name__ == "__main__":
    download_data("data/all_data.zip")
