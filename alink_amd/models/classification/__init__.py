"""Classification models beyond the linear family: naive Bayes (text), MLP, FM, one-vs-rest."""
