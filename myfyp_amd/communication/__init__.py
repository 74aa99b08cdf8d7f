"""Communication: commands (control + weights messages) and transport protocols."""
