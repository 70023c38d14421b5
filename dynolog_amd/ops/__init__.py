"""dynolog_amd.ops"""
