"""Front-end helpers for the Streamlit client (reference: src/streamlit_ui/cobalt_streamlit.py)."""
