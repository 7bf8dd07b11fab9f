"""NN challenger (notebook 04): fused MLP trainer/inference, SMOTE, MinMaxScaler."""
