"""Streamlit front end (reference: src/streamlit_ui/cobalt_streamlit.py).

Two modes: a single-borrower form posting to /predict and showing the probability plus a SHAP
waterfall, and a CSV upload posting to /predict_bulk_csv with a results table, CSV download and the
top-10 gain-importance chart from /feature_importance_bulk. All request/plot logic lives in
``cobalt_smart_lender_ai_amd.ui.client`` (unit-tested without Streamlit); this file only lays out
widgets. ``API_URL`` comes from the environment (default ``http://cobalt-lender-api:8000``).

Run: ``streamlit run src/streamlit_ui/cobalt_streamlit.py``
"""
import io
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import pandas as pd  # noqa: E402
import streamlit as st  # noqa: E402

from cobalt_smart_lender_ai_amd.ui import client as ui  # noqa: E402

api = ui.ApiClient()
st.set_page_config(page_title="Cobalt Loan Default Prediction", layout="wide")
st.title("Loan Default Risk Predictor")
menu = st.sidebar.radio("Select Mode", ["Single Prediction", "Bulk Prediction + SHAP"])

if menu == "Single Prediction":
    st.subheader("Enter loan details for a single borrower")
    c1, c2 = st.columns(2)
    num = {}
    with c1:
        num["loan_amnt"] = st.number_input("Loan Amount", value=10000.0, min_value=0.0)
        num["term"] = st.selectbox("Term (months)", [36, 60], index=0)
        num["installment"] = st.number_input("Installment", value=300.0)
        num["fico_range_low"] = st.number_input("FICO Range Low", value=660.0)
        num["last_fico_range_high"] = st.number_input("Last FICO High", value=700.0)
        num["open_il_12m"] = st.number_input("Open IL Last 12m", value=1.0)
        num["open_il_24m"] = st.number_input("Open IL Last 24m", value=2.0)
    with c2:
        num["max_bal_bc"] = st.number_input("Max Balance on Bank Card", value=2000.0)
        num["num_rev_accts"] = st.number_input("Number of Revolving Accounts", value=10.0)
        num["pub_rec_bankruptcies"] = st.number_input("Bankruptcies", value=0.0)
        num["emp_length_num"] = st.number_input("Employment Length (years)", value=3.0)
        num["earliest_cr_line_days"] = st.number_input("Days Since First Credit Line", value=4000.0)
        g = st.checkbox("Grade E")
        m = st.checkbox("Home Ownership: Mortgage")
        v = st.checkbox("Verified Status")
        j = st.checkbox("Joint Application")
        h = st.selectbox("Hardship Status", ui.HARDSHIP_CHOICES)
    payload = ui.single_payload(num, g, m, v, j, h)
    if st.button("Predict Default Risk"):
        try:
            r = api.predict(payload)
            st.success(f"Estimated Default Probability: {r['prob_default']:.2%}")
            st.subheader("SHAP Explanation")
            fig = ui.waterfall_figure(r["shap_values"], r["base_value"],
                                      [r["input_row"][f] for f in r["features"]], r["features"])
            st.pyplot(fig)
        except Exception as e:  # surfaced in the page, as the reference does
            st.error(f"Error during prediction: {e}")
else:
    st.subheader("Upload CSV for Bulk Inference")
    up = st.file_uploader("Upload CSV with required columns", type="csv")
    if up:
        try:
            df = pd.read_csv(io.BytesIO(up.getvalue()))
            st.write("Uploaded Data Preview:", df.head())
        except Exception as e:
            st.error(f"Failed to read CSV: {e}")
            st.stop()
        if st.button("Run Bulk Prediction"):
            try:
                rows = api.predict_bulk_csv(up.name, up.getvalue())
                out = pd.DataFrame(rows).apply(pd.to_numeric, errors="coerce")
                st.subheader("Prediction Results")
                st.dataframe(out)
                st.download_button("Download Results", out.to_csv(index=False), "bulk_predictions.csv")
                st.subheader("Feature Importance (Top 10)")
                st.pyplot(ui.importance_figure(api.feature_importance_bulk(rows)))
            except Exception as e:
                st.error(f"Bulk prediction failed: {e}")
