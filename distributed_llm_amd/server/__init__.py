"""server"""
