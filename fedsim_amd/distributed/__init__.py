"""Distributed (federated) learning on the MI355X aggregation path."""
