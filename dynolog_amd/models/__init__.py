"""dynolog_amd.models"""
