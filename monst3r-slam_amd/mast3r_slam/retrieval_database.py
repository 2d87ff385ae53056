"""mast3r_slam.retrieval_database (retrieval_database.py:9-166) with the device-resident
inverted file."""
from monst3r_slam_amd.retrieval import RetrievalDatabase, load_retriever  # noqa: F401
